// Host JPEG entropy decoder throughput vs thread count (csrc/host/jpeg_decode.cpp).
// g++ -O3 -std=c++17 -pthread -I lumen_amd/csrc/host -I lumen_amd/csrc tools/probes/jd_probe.cpp \
//     lumen_amd/csrc/host/jpeg_decode.cpp -o /tmp/jd_probe && /tmp/jd_probe
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <fstream>
#include <iterator>
#include <vector>
extern "C" int lumen_jpeg_decode_coefs(const uint8_t*, uint64_t, int, int16_t*, uint16_t*, int64_t*);
int main() {
  std::ifstream f("tools/probes/photo_probe.jpg", std::ios::binary);
  std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), {});
  static int16_t coefs[4 << 20]; uint16_t qt[256]; int64_t st[4];
  for (int th : {1, 4, 8, 12, 16}) {
    for (int i = 0; i < 5; i++) lumen_jpeg_decode_coefs(d.data(), d.size(), th, coefs, qt, st);
    auto t0 = std::chrono::steady_clock::now(); const int N = 30;
    for (int i = 0; i < N; i++) lumen_jpeg_decode_coefs(d.data(), d.size(), th, coefs, qt, st);
    printf("threads %d: %.0f us per 1024x768 photo (chunks %ld)\n", th,
           std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / N, (long)st[0]);
  }
}
