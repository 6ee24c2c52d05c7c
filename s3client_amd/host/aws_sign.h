// aws_sign.h -- SigV4 signing that CONSUMES the payload digest (parity harness, config 1).
//
// Restates the reference signer's observable behaviour (lib/src/aws_sign.cpp:226-325
// ComputeSignature / SignHeaders, :130-221 SignedURL; config structs lib/include/aws_sign.h)
// on top of the lib/hash drop-in (include/sha256.h: sha256::sha256, hmac256).  It exists so
// the build can show, end to end, that a GPU payload digest slots into
// `x-amz-content-sha256` exactly where the reference puts "UNSIGNED-PAYLOAD"
// (aws_sign.cpp:236-237).  Own code; field names follow the reference's config structs.
#pragma once
#include <map>
#include <string>

namespace s3h {
namespace sigv4 {

using Map = std::map<std::string, std::string>;  // sorted, like sss::Map (common.h:54)

struct Dates {
  std::string timeStamp;  // "%Y%m%dT%H%M%SZ"
  std::string dateStamp;  // "%Y%m%d"
};

struct SignConfig {  // mirrors sss::ComputeSignatureConfig (aws_sign.h:67-80)
  std::string access, secret, endpoint, method, bucket, key;
  std::string payloadHash;  // empty -> "UNSIGNED-PAYLOAD"
  Map parameters;
  Map headers;
  std::string region = "us-east";
  std::string service = "s3";
  Dates dates;  // empty dateStamp -> current UTC time
};

struct PresignConfig {  // mirrors sss::S3SignUrlConfig (aws_sign.h:83-95)
  std::string access, secret, endpoint;
  int expiration = 0;
  std::string method, bucket, key;
  Map params;
  Map headers;
  std::string region = "us-east";
  Dates dates;
};

struct Signature {
  std::string signature, credentialScope, signedHeadersStr;
  Map defaultHeaders;
};

std::string UrlEncode(const std::string& s);
std::string UrlEncode(const Map& m);
std::string Sha256Hex(const std::string& s);  // lowercase hex digest (CPU drop-in)

Signature ComputeSignature(const SignConfig& cfg);
Map SignHeaders(const SignConfig& cfg);
std::string SignedURL(const PresignConfig& cfg);

}  // namespace sigv4
}  // namespace s3h
