// Host-runtime stress driver for the sanitizer test (tests/test_host_sanitizers.py):
// exercises the DB-net geometry, the similarity transform and the paged-KV block
// manager (from 4 threads concurrently) so ASan/UBSan/TSan see every code path.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

extern "C" {
int lumen_db_boxes(const float* prob, int H, int W, float thresh, float box_thresh, float unclip_ratio,
                   int max_candidates, int min_size, float scale_x, float scale_y, int src_w, int src_h,
                   float* boxes, float* scores, int max_boxes);
void lumen_similarity_transform(const float* src, const float* dst, int n, float* M);
void* lumen_kv_create(int num_blocks);
void lumen_kv_destroy(void* h);
int lumen_kv_reserve(void* h, int64_t seq, int n_tokens);
int lumen_kv_table(void* h, int64_t seq, int* out, int max);
int lumen_kv_fork(void* h, int64_t src, int64_t dst);
int lumen_kv_release(void* h, int64_t seq);
int lumen_kv_free_blocks(void* h);
}

int main() {
  // geometry: a few rectangles + noise on a 120x160 map
  const int H = 120, W = 160;
  std::vector<float> prob(H * W, 0.f);
  for (int r = 0; r < 4; ++r)
    for (int y = 10 + 25 * r; y < 22 + 25 * r; ++y)
      for (int x = 8 + 10 * r; x < 90 + 12 * r && x < W; ++x) prob[y * W + x] = 0.9f;
  unsigned s = 1;
  for (int i = 0; i < H * W; ++i) { s = s * 1103515245u + 12345u; if ((s >> 16) % 97 == 0) prob[i] = 0.8f; }
  std::vector<float> boxes(64 * 8), scores(64);
  const int n = lumen_db_boxes(prob.data(), H, W, 0.3f, 0.5f, 1.5f, 1000, 3, 2.f, 2.f, 320, 240, boxes.data(),
                               scores.data(), 64);
  if (n < 4) { std::fprintf(stderr, "expected >= 4 boxes, got %d\n", n); return 1; }
  const float src[10] = {50, 60, 90, 58, 70, 80, 55, 100, 88, 99};
  const float dst[10] = {38.29f, 51.69f, 73.53f, 51.5f, 56.02f, 71.73f, 41.54f, 92.36f, 70.72f, 92.2f};
  float M[6];
  lumen_similarity_transform(src, dst, 5, M);
  if (!std::isfinite(M[0])) return 2;
  // block manager under concurrency
  void* h = lumen_kv_create(256);
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([h, t] {
      int tab[64];
      for (int i = 0; i < 2000; ++i) {
        const int64_t seq = t * 100000 + i;
        if (lumen_kv_reserve(h, seq, 1 + (i * 37) % 500) >= 0) {
          lumen_kv_table(h, seq, tab, 64);
          if (i % 3 == 0) { lumen_kv_fork(h, seq, seq + 50000); lumen_kv_release(h, seq + 50000); }
          lumen_kv_release(h, seq);
        }
        lumen_kv_free_blocks(h);
      }
    });
  for (auto& x : th) x.join();
  const int free_blocks = lumen_kv_free_blocks(h);
  lumen_kv_destroy(h);
  if (free_blocks != 256) { std::fprintf(stderr, "leaked blocks: %d free\n", free_blocks); return 3; }
  std::printf("ok boxes=%d\n", n);
  return 0;
}
