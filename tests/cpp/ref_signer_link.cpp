// tests/cpp/ref_signer_link.cpp -- link proof for the drop-in boundary.
//
// The reference's OWN signer translation units -- /root/reference/lib/src/aws_sign.cpp,
// url_utility.cpp and utility.cpp, compiled unmodified from where they lie (recipe:
// oracle/Makefile target `refsigner`) with this repo's include/sha256.h + utility.h in place
// of lib/hash's -- are linked against libs3hash.so instead of lib/hash/*.cpp.  aws_sign.o
// imports exactly sha256::sha256 and hmac256 (nm -u), which must resolve to the drop-in.
// This driver replays the reference's signer known-answer tests through them:
//   test/sign-test.cpp:43-57         -> "Sign,Sign request,1,"
//   test/presign-url-test.cpp:11-27  -> "Sign,Presign URL,1"
// plus the same request signed with a real payload digest.
// (The reference's test mains themselves include s3-client.h -> webclient.h -> <curl/curl.h>,
// whose headers this image lacks, so the KAT configs are restated here; no stand-in headers.)
#include <iostream>
#include <string>

#include "aws_sign.h"  // the reference's lib/include/aws_sign.h
#include "sha256.h"    // this repo's drop-in header

using namespace sss;

int main() {
  int fails = 0;
  const ComputeSignatureConfig cfg{.access = "08XW32=0H=G7=HBLCG",
                                   .secret = "y8a=4KnHBxTtOuH5zduTxjfFIjBXfwfBWfjF",
                                   .endpoint = "http://localhost:9000",
                                   .method = "GET",
                                   .bucket = "bucket1",
                                   .key = "key1",
                                   .headers = {{"x-amz-meta-mymeta", "123"}},
                                   .dates = {"20230418T153022Z", "20230418"}};
  const bool sign_ok = ComputeSignature(cfg).signature ==
                       "2ff4da4766da392b60b3278d2993398ee3f05fbf45aae378a66b489d266a4e87";
  std::cout << "Sign," << "Sign request," << sign_ok << ',' << std::endl;
  fails += !sign_ok;

  const S3SignUrlConfig pcfg{.access = "7PJRLUIHCX+/1O63TN",
                             .secret = "bTDYuxv+0teEVY9gUYWM7p3B3x=GuiFAtO+4",
                             .endpoint = "http://127.0.0.1:9000",
                             .expiration = 1000,
                             .method = "PUT",
                             .bucket = "bucket1",
                             .key = "key1",
                             .dates = {"20230418T153022Z", "20230418"}};
  const bool url_ok =
      SignedURL(pcfg) ==
      "http://127.0.0.1:9000/bucket1/"
      "key1?X-Amz-Algorithm=AWS4-HMAC-SHA256&X-Amz-Credential=7PJRLUIHCX%2B%"
      "2F1O63TN%2F20230418%2Fus-east%2Fs3%2Faws4_request&X-Amz-Date="
      "20230418T153022Z&X-Amz-Expires=1000&X-Amz-SignedHeaders=host&X-Amz-"
      "Signature=e48f7576e8978074bb747f4cfed31230da726cce9074ef577a9739149c4d342a";
  std::cout << "Sign," << "Presign URL," << url_ok << std::endl;
  fails += !url_ok;

  // PUT carrying x-amz-content-sha256 = the drop-in's digest of "12345678" x 6
  std::string body;
  for (int i = 0; i < 6; ++i) body += "12345678";
  uint32_t h[8];
  sha256::sha256(reinterpret_cast<const uint8_t*>(body.data()), body.size(), h);
  char hex[65];
  sha256::hash_to_text(h, hex);
  ComputeSignatureConfig put = cfg;
  put.method = "PUT";
  put.payloadHash = hex;
  const Signature ps = ComputeSignature(put);
  const bool pay_ok = ps.signature == "3c1ee8b1e795824dedfe3d0271f070291523022c94fbd39ff559079d776296d1" &&
                      ps.signedHeadersStr == "host;x-amz-content-sha256;x-amz-date;x-amz-meta-mymeta";
  std::cout << "Sign," << "Sign payload request," << pay_ok << ',' << std::endl;
  fails += !pay_ok;
  return fails ? 1 : 0;
}
