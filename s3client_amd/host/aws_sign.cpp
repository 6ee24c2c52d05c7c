// aws_sign.cpp -- see aws_sign.h.  Behaviour follows /root/reference/lib/src/aws_sign.cpp
// (cited per function); hashing goes through the lib/hash drop-in in libs3hash.so.
#include "aws_sign.h"

#include <cctype>
#include <cstdint>
#include <ctime>
#include <regex>
#include <set>
#include <string>
#include <vector>

#include "sha256.h"

namespace s3h {
namespace sigv4 {
namespace {

using Bytes = std::vector<uint8_t>;

const char kHex[] = "0123456789abcdef";

std::string hex(const uint8_t* p, size_t n) {
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    s[2 * i] = kHex[p[i] >> 4];
    s[2 * i + 1] = kHex[p[i] & 15];
  }
  return s;
}

Bytes hmac(const Bytes& key, const std::string& msg) {  // aws_sign.cpp:71-75, 98
  Bytes out(32);
  hmac256(reinterpret_cast<const uint8_t*>(msg.data()), msg.size(), key.data(), key.size(),
          out.data());
  return out;
}

// SigV4 signing key: HMAC chain over date, region, service, "aws4_request" (aws_sign.cpp:102-113)
Bytes signing_key(const std::string& secret, const std::string& date, const std::string& region,
                  const std::string& service) {
  const std::string k = "AWS4" + secret;
  Bytes key(k.begin(), k.end());
  for (const std::string* part : {&date, &region, &service}) key = hmac(key, *part);
  return hmac(key, "aws4_request");
}

struct HostPort {
  std::string host;
  int port = -1;
};

// {proto}://{host}[:{port}] (url_utility.cpp:51-66)
HostPort parse_url(const std::string& url) {
  static const std::regex re(R"(\s*(\w+)://([0-9a-zA-Z\-_\.]+)(:(\d+))?)");
  std::smatch m;
  HostPort hp;
  if (!std::regex_search(url, m, re)) return hp;
  hp.host = m[2];
  if (m[4].matched && !m[4].str().empty()) hp.port = std::stoi(m[4]);
  return hp;
}

std::string host_header(const std::string& endpoint) {
  const HostPort hp = parse_url(endpoint);
  return hp.port <= 0 ? hp.host : hp.host + ":" + std::to_string(hp.port);
}

Dates now_dates() {  // aws_sign.cpp:80-94
  std::time_t t = std::time(nullptr);
  std::tm tm{};
  gmtime_r(&t, &tm);
  char a[32], b[32];
  std::strftime(a, sizeof a, "%Y%m%dT%H%M%SZ", &tm);
  std::strftime(b, sizeof b, "%Y%m%d", &tm);
  return {a, b};
}

std::string upper(std::string s) {
  for (auto& c : s) c = char(std::toupper(static_cast<unsigned char>(c)));
  return s;
}

std::string resource(const std::string& bucket, const std::string& key) {
  std::string r = "/";
  if (!bucket.empty()) {
    r += bucket;
    if (!key.empty()) r += "/" + key;
  }
  return r;
}

bool starts_with(const std::string& s, const char* p) { return s.rfind(p, 0) == 0; }

}  // namespace

std::string UrlEncode(const std::string& s) {  // url_utility.cpp:70-90
  static const char kUp[] = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      o += char(c);
    } else {
      o += '%';
      o += kUp[c >> 4];
      o += kUp[c & 15];
    }
  }
  return o;
}

std::string UrlEncode(const Map& m) {  // url_utility.cpp:93-100 (key=value joined by '&')
  std::string o;
  for (const auto& kv : m) {
    if (!o.empty()) o += '&';
    o += UrlEncode(kv.first) + "=" + UrlEncode(kv.second);
  }
  return o;
}

std::string Sha256Hex(const std::string& s) {  // sss::SHA256, aws_sign.cpp:63-69
  uint32_t h[8];
  sha256::sha256(reinterpret_cast<const uint8_t*>(s.data()), s.size(), h);
  char t[65];
  sha256::hash_to_text(h, t);
  return t;
}

Signature ComputeSignature(const SignConfig& cfg) {  // aws_sign.cpp:226-308
  const std::string payload = cfg.payloadHash.empty() ? "UNSIGNED-PAYLOAD" : cfg.payloadHash;
  const Dates d = cfg.dates.dateStamp.empty() ? now_dates() : cfg.dates;
  Signature sig;
  sig.defaultHeaders = {{"host", host_header(cfg.endpoint)},
                        {"x-amz-content-sha256", payload},
                        {"x-amz-date", d.timeStamp}};
  Map canonical = sig.defaultHeaders;
  for (const auto& kv : cfg.headers)  // x-amz-* and content-length are signed (:266-271)
    if (starts_with(kv.first, "x-amz-") || starts_with(kv.first, "content-length"))
      canonical.insert(kv);
  std::string headers_block, signed_list;
  for (const auto& kv : canonical) {
    headers_block += kv.first + ":" + kv.second + "\n";
    signed_list += (signed_list.empty() ? "" : ";") + kv.first;
  }
  const std::string query = cfg.parameters.empty() ? "" : UrlEncode(cfg.parameters);
  const std::string request = upper(cfg.method) + "\n" + resource(cfg.bucket, cfg.key) + "\n" +
                              query + "\n" + headers_block + "\n" + signed_list + "\n" + payload;
  sig.credentialScope = d.dateStamp + "/" + cfg.region + "/" + cfg.service + "/aws4_request";
  const std::string to_sign = "AWS4-HMAC-SHA256\n" + d.timeStamp + "\n" + sig.credentialScope +
                              "\n" + Sha256Hex(request);
  const Bytes mac = hmac(signing_key(cfg.secret, d.dateStamp, cfg.region, cfg.service), to_sign);
  sig.signature = hex(mac.data(), mac.size());
  sig.signedHeadersStr = signed_list;
  return sig;
}

Map SignHeaders(const SignConfig& cfg) {  // aws_sign.cpp:313-325
  const Signature s = ComputeSignature(cfg);
  Map all = s.defaultHeaders;
  all.insert({"Authorization", "AWS4-HMAC-SHA256 Credential=" + cfg.access + "/" +
                                   s.credentialScope + ", SignedHeaders=" + s.signedHeadersStr +
                                   ", Signature=" + s.signature});
  all.insert(cfg.headers.begin(), cfg.headers.end());
  return all;
}

std::string SignedURL(const PresignConfig& cfg) {  // aws_sign.cpp:130-221
  const std::string host = host_header(cfg.endpoint);
  const Dates d = cfg.dates.dateStamp.empty() ? now_dates() : cfg.dates;
  // The reference adds to the signed set the headers that do NOT start with "x-amz-"
  // (`find("x-amz-")` is truthy unless the match is at position 0, aws_sign.cpp:148).
  Map signed_headers = {{"host", host}};
  for (const auto& kv : cfg.headers)
    if (!starts_with(kv.first, "x-amz-")) signed_headers.insert(kv);
  std::string signed_list;
  for (const auto& kv : signed_headers) signed_list += (signed_list.empty() ? "" : ";") + kv.first;
  Map all_headers = cfg.headers;
  all_headers.insert({"host", host});
  std::string headers_block;
  for (const auto& kv : all_headers) headers_block += kv.first + ":" + kv.second + "\n";
  Map params = {{"X-Amz-Algorithm", "AWS4-HMAC-SHA256"},
                {"X-Amz-Credential", cfg.access + "/" + d.dateStamp + "/" + cfg.region +
                                         "/s3/aws4_request"},
                {"X-Amz-Date", d.timeStamp},
                {"X-Amz-Expires", std::to_string(cfg.expiration)},
                {"X-Amz-SignedHeaders", signed_list}};
  params.insert(cfg.params.begin(), cfg.params.end());
  const std::string query = UrlEncode(params);
  const std::string res = resource(cfg.bucket, cfg.key);
  const std::string request = cfg.method + "\n" + res + "\n" + query + "\n" + headers_block +
                              "\n" + signed_list + "\nUNSIGNED-PAYLOAD";
  const std::string scope = d.dateStamp + "/" + cfg.region + "/s3/aws4_request";
  const std::string to_sign =
      "AWS4-HMAC-SHA256\n" + d.timeStamp + "\n" + scope + "\n" + Sha256Hex(request);
  const Bytes mac = hmac(signing_key(cfg.secret, d.dateStamp, cfg.region, "s3"), to_sign);
  std::string url = cfg.endpoint;
  if (!cfg.bucket.empty()) {
    url += "/" + cfg.bucket;
    if (!cfg.key.empty()) url += "/" + cfg.key;
  }
  return url + "?" + query + "&X-Amz-Signature=" + hex(mac.data(), mac.size());
}

}  // namespace sigv4
}  // namespace s3h
