// Host-side geometry for DB-net text detection post-processing (C ABI, ctypes).
//
// Replaces the OpenCV / pyclipper / shapely calls of the reference
// (packages/lumen-ocr/src/lumen_ocr/backends/onnxrt_backend.py:380-476:
// cv2.findContours, cv2.minAreaRect, box_score_fast, pyclipper unclip):
//   1. connected components of the thresholded probability bitmap (8-connected,
//      union-find, two passes), one component = one contour candidate;
//   2. per component: convex hull (Andrew monotone chain) of the pixel centres,
//      minimum-area rectangle by rotating calipers over hull edges
//      (== cv2.minAreaRect of the outer contour);
//   3. box score = mean probability inside the rectangle (box_score_fast);
//   4. unclip: distance d = area * ratio / perimeter; a rectangle offset by d with
//      round joins has the rectangle grown by d per side as its min-area rect;
//   5. size filters, clockwise TL,TR,BR,BL ordering, rescale to the source image.
// Runs on CPU threads next to the GPU (the bitmap is small: <= 960x960).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <climits>
#include <numeric>
#include <vector>

namespace {

struct P { double x, y; };

double cross(const P& o, const P& a, const P& b) { return (a.x - o.x) * (b.y - o.y) - (a.y - o.y) * (b.x - o.x); }

std::vector<P> hull(std::vector<P> pts) {
  std::sort(pts.begin(), pts.end(), [](const P& a, const P& b) { return a.x < b.x || (a.x == b.x && a.y < b.y); });
  pts.erase(std::unique(pts.begin(), pts.end(), [](const P& a, const P& b) { return a.x == b.x && a.y == b.y; }),
            pts.end());
  if (pts.size() < 3) return pts;
  std::vector<P> h(2 * pts.size());
  size_t k = 0;
  for (size_t i = 0; i < pts.size(); ++i) {
    while (k >= 2 && cross(h[k - 2], h[k - 1], pts[i]) <= 0) --k;
    h[k++] = pts[i];
  }
  for (size_t i = pts.size() - 1, t = k + 1; i > 0; --i) {
    while (k >= t && cross(h[k - 2], h[k - 1], pts[i - 1]) <= 0) --k;
    h[k++] = pts[i - 1];
  }
  h.resize(k - 1);
  return h;
}

// minimum-area rectangle of a convex polygon: centre, (w, h), angle
struct Rect { double cx, cy, w, h, ang; };

Rect min_area_rect(const std::vector<P>& h) {
  Rect best{0, 0, 0, 0, 0};
  if (h.empty()) return best;
  if (h.size() == 1) return Rect{h[0].x, h[0].y, 0, 0, 0};
  if (h.size() == 2) {
    const double dx = h[1].x - h[0].x, dy = h[1].y - h[0].y;
    return Rect{(h[0].x + h[1].x) / 2, (h[0].y + h[1].y) / 2, std::sqrt(dx * dx + dy * dy), 0, std::atan2(dy, dx)};
  }
  double best_area = 1e300;
  const size_t n = h.size();
  for (size_t i = 0; i < n; ++i) {
    const P& a = h[i];
    const P& b = h[(i + 1) % n];
    double ux = b.x - a.x, uy = b.y - a.y;
    const double len = std::sqrt(ux * ux + uy * uy);
    if (len < 1e-12) continue;
    ux /= len; uy /= len;
    const double vx = -uy, vy = ux;
    double mnu = 1e300, mxu = -1e300, mnv = 1e300, mxv = -1e300;
    for (const P& p : h) {
      const double pu = p.x * ux + p.y * uy, pv = p.x * vx + p.y * vy;
      mnu = std::min(mnu, pu); mxu = std::max(mxu, pu);
      mnv = std::min(mnv, pv); mxv = std::max(mxv, pv);
    }
    const double area = (mxu - mnu) * (mxv - mnv);
    if (area < best_area) {
      best_area = area;
      const double cu = (mnu + mxu) / 2, cv = (mnv + mxv) / 2;
      best = Rect{cu * ux + cv * vx, cu * uy + cv * vy, mxu - mnu, mxv - mnv, std::atan2(uy, ux)};
    }
  }
  return best;
}

void rect_corners(const Rect& r, P out[4]) {
  const double c = std::cos(r.ang), s = std::sin(r.ang);
  const double hw = r.w / 2, hh = r.h / 2;
  const double dx[4] = {-hw, hw, hw, -hw}, dy[4] = {-hh, -hh, hh, hh};
  for (int i = 0; i < 4; ++i) out[i] = P{r.cx + dx[i] * c - dy[i] * s, r.cy + dx[i] * s + dy[i] * c};
}

// order clockwise starting top-left (reference get_mini_boxes ordering)
void order_box(P b[4]) {
  std::sort(b, b + 4, [](const P& a, const P& c) { return a.x < c.x; });
  P tl, bl, tr, br;
  if (b[0].y <= b[1].y) { tl = b[0]; bl = b[1]; } else { tl = b[1]; bl = b[0]; }
  if (b[2].y <= b[3].y) { tr = b[2]; br = b[3]; } else { tr = b[3]; br = b[2]; }
  b[0] = tl; b[1] = tr; b[2] = br; b[3] = bl;
}

bool in_quad(const P q[4], double x, double y) {
  bool pos = false, neg = false;
  for (int i = 0; i < 4; ++i) {
    const double c = cross(q[i], q[(i + 1) % 4], P{x, y});
    if (c > 0) pos = true;
    if (c < 0) neg = true;
  }
  return !(pos && neg);
}

int find(std::vector<int>& p, int x) {
  while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; }
  return x;
}

}  // namespace

extern "C" {

// prob: float [H, W]; bitmap from (prob > thresh).  Output up to max_boxes boxes:
// boxes[i*8 .. +8] = 4 (x, y) corners (clockwise from TL) in source-image pixels,
// scores[i].  Returns the number of boxes.
int lumen_db_boxes(const float* prob, int H, int W, float thresh, float box_thresh, float unclip_ratio,
                   int max_candidates, int min_size, float scale_x, float scale_y, int src_w, int src_h,
                   float* boxes, float* scores, int max_boxes) {
  const int n = H * W;
  std::vector<int> lab(n, -1);
  std::vector<int> parent;
  parent.reserve(1024);
  for (int y = 0; y < H; ++y) {
    for (int x = 0; x < W; ++x) {
      const int i = y * W + x;
      if (!(prob[i] > thresh)) continue;
      int best = -1;
      const int nb[4][2] = {{-1, 0}, {-1, -1}, {0, -1}, {1, -1}};  // W, NW, N, NE
      for (auto& d : nb) {
        const int xx = x + d[0], yy = y + d[1];
        if (xx < 0 || yy < 0 || xx >= W) continue;
        const int l = lab[yy * W + xx];
        if (l < 0) continue;
        if (best < 0) best = find(parent, l);
        else {
          const int a = find(parent, l), b = best;
          if (a != b) parent[std::max(a, b)] = std::min(a, b), best = std::min(a, b);
        }
      }
      if (best < 0) { best = (int)parent.size(); parent.push_back(best); }
      lab[i] = best;
    }
  }
  const int ncomp = (int)parent.size();
  std::vector<int> root(ncomp);
  for (int c = 0; c < ncomp; ++c) root[c] = find(parent, c);
  std::vector<int> remap(ncomp, -1);
  int nroots = 0;
  for (int c = 0; c < ncomp; ++c)
    if (root[c] == c) remap[c] = nroots++;
  std::vector<std::vector<P>> pts(nroots);
  for (int i = 0; i < n; ++i) {
    if (lab[i] < 0) continue;
    const int c = remap[root[lab[i]]];
    // boundary pixels only (any 4-neighbour outside) keeps hulls cheap
    const int x = i % W, y = i / W;
    const bool interior = x > 0 && y > 0 && x < W - 1 && y < H - 1 && lab[i - 1] >= 0 && lab[i + 1] >= 0 &&
                          lab[i - W] >= 0 && lab[i + W] >= 0;
    if (!interior) pts[c].push_back(P{(double)x, (double)y});
  }
  int out = 0;
  const int ncand = std::min(nroots, max_candidates);
  for (int c = 0; c < ncand && out < max_boxes; ++c) {
    if (pts[c].size() < 3) continue;
    const std::vector<P> h = hull(pts[c]);
    Rect r = min_area_rect(h);
    if (std::min(r.w, r.h) < min_size) continue;
    P q[4];
    rect_corners(r, q);
    // box score: mean prob inside the rectangle
    double xmin = 1e9, xmax = -1e9, ymin = 1e9, ymax = -1e9;
    for (auto& p : q) { xmin = std::min(xmin, p.x); xmax = std::max(xmax, p.x); ymin = std::min(ymin, p.y); ymax = std::max(ymax, p.y); }
    const int x0 = std::max(0, (int)std::floor(xmin)), x1 = std::min(W - 1, (int)std::ceil(xmax));
    const int y0 = std::max(0, (int)std::floor(ymin)), y1 = std::min(H - 1, (int)std::ceil(ymax));
    double s = 0;
    int cnt = 0;
    for (int yy = y0; yy <= y1; ++yy)
      for (int xx = x0; xx <= x1; ++xx)
        if (in_quad(q, xx, yy)) { s += prob[yy * W + xx]; ++cnt; }
    const double score = cnt ? s / cnt : 0.0;
    if (score < box_thresh) continue;
    // unclip: grow by d = area * ratio / perimeter on each side
    const double area = r.w * r.h, perim = 2 * (r.w + r.h);
    const double d = perim > 0 ? area * unclip_ratio / perim : 0;
    r.w += 2 * d;
    r.h += 2 * d;
    if (std::min(r.w, r.h) < min_size + 2) continue;
    rect_corners(r, q);
    order_box(q);
    for (int k = 0; k < 4; ++k) {
      const double X = std::min(std::max(std::round(q[k].x * scale_x), 0.0), (double)src_w);
      const double Y = std::min(std::max(std::round(q[k].y * scale_y), 0.0), (double)src_h);
      boxes[out * 8 + 2 * k] = (float)X;
      boxes[out * 8 + 2 * k + 1] = (float)Y;
    }
    scores[out] = (float)score;
    ++out;
  }
  return out;
}

// ---- split form for the GPU labelling path (csrc/db_post.hip) ----------------------------
// pts: int32 [K, 3] rows (root, x, y) as the GPU appended them (atomic order) -> sorted by root in
// place, stable (LSD radix sort, 12-bit digits, passes for the largest root only): replaces a
// device radix sort + gather + copy (torch.sort) between the labelling kernels and the D2H.
void lumen_sort_points_by_root(int* pts, int K) {
  if (K < 2) return;
  int maxk = 0;
  for (int i = 0; i < K; ++i) maxk = std::max(maxk, pts[3 * i]);
  // (key, row) pairs sorted on 12-bit digits (2 passes for the < 2^24 pixel indices of a 16-map
  // batch, 3 at most: shift < 32 also keeps `maxk >> shift` defined), then one gather of the 12-byte rows
  std::vector<uint64_t> a((size_t)K), b((size_t)K);
  for (int i = 0; i < K; ++i) a[i] = ((uint64_t)(uint32_t)pts[3 * i] << 32) | (uint32_t)i;
  std::vector<int> cnt(4096);
  for (int shift = 0; shift < 32 && (shift == 0 || (maxk >> shift) > 0); shift += 12) {
    std::fill(cnt.begin(), cnt.end(), 0);
    for (int i = 0; i < K; ++i) ++cnt[(a[i] >> (32 + shift)) & 4095];
    int run = 0;
    for (int d = 0; d < 4096; ++d) {
      const int c = cnt[d];
      cnt[d] = run;
      run += c;
    }
    for (int i = 0; i < K; ++i) b[cnt[(a[i] >> (32 + shift)) & 4095]++] = a[i];
    a.swap(b);
  }
  std::vector<int> rows((size_t)3 * K);
  for (int i = 0; i < K; ++i) {
    const uint32_t r = (uint32_t)(a[i] & 0xffffffffu);
    rows[3 * i] = pts[3 * r];
    rows[3 * i + 1] = pts[3 * r + 1];
    rows[3 * i + 2] = pts[3 * r + 2];
  }
  std::memcpy(pts, rows.data(), sizeof(int) * 3 * (size_t)K);
}

// pts: int32 [K, 3] boundary pixels (component root, x, y) grouped by root in ascending
// root order (== the raster order of the components' first pixels, as above).  For the
// first max_candidates components: hull -> min-area rect; rects below min_size dropped.
// Writes quads [n, 8] (the rect's corners, for the GPU box score), rects [n, 5]
// (cx, cy, w, h, angle) and the component root; returns n.
int lumen_db_candidates(const int* pts, int K, int max_candidates, int min_size, float* quads, float* rects,
                        int* roots, int max_out) {
  int out = 0, comps = 0;
  for (int i = 0; i < K && out < max_out;) {
    int j = i;
    while (j < K && pts[3 * j] == pts[3 * i]) ++j;
    if (comps++ >= max_candidates) break;
    if (j - i >= 3) {
      // the hull of a pixel set is the hull of each row's leftmost / rightmost pixel: reduce a
      // large component's boundary (an untrained map's blob: ~10^5 pixels) to <= 2 per row in O(n)
      int ymin = pts[3 * i + 2], ymax = ymin;
      for (int t = i; t < j; ++t) { ymin = std::min(ymin, pts[3 * t + 2]); ymax = std::max(ymax, pts[3 * t + 2]); }
      std::vector<int> lo(ymax - ymin + 1, INT32_MAX), hi(ymax - ymin + 1, INT32_MIN);
      for (int t = i; t < j; ++t) {
        const int yy = pts[3 * t + 2] - ymin, xx = pts[3 * t + 1];
        lo[yy] = std::min(lo[yy], xx);
        hi[yy] = std::max(hi[yy], xx);
      }
      std::vector<P> v;
      v.reserve(2 * lo.size());
      for (size_t yy = 0; yy < lo.size(); ++yy) {
        if (lo[yy] == INT32_MAX) continue;
        v.push_back(P{(double)lo[yy], (double)(yy + ymin)});
        if (hi[yy] != lo[yy]) v.push_back(P{(double)hi[yy], (double)(yy + ymin)});
      }
      const Rect r = min_area_rect(hull(v));
      if (std::min(r.w, r.h) >= min_size) {
        P q[4];
        rect_corners(r, q);
        for (int k = 0; k < 4; ++k) { quads[out * 8 + 2 * k] = (float)q[k].x; quads[out * 8 + 2 * k + 1] = (float)q[k].y; }
        const double rv[5] = {r.cx, r.cy, r.w, r.h, r.ang};
        for (int k = 0; k < 5; ++k) rects[out * 5 + k] = (float)rv[k];
        roots[out] = pts[3 * i];
        ++out;
      }
    }
    i = j;
  }
  return out;
}

// score filter, unclip, size filter, TL-clockwise order, rescale + clip (lumen_db_boxes steps 3b-5)
int lumen_db_finalize(const float* rects, const float* scores, int m, float box_thresh, float unclip_ratio,
                      int min_size, float scale_x, float scale_y, int src_w, int src_h, float* boxes,
                      float* out_scores, int max_boxes) {
  int out = 0;
  for (int i = 0; i < m && out < max_boxes; ++i) {
    if (scores[i] < box_thresh) continue;
    Rect r{rects[i * 5], rects[i * 5 + 1], rects[i * 5 + 2], rects[i * 5 + 3], rects[i * 5 + 4]};
    const double area = r.w * r.h, perim = 2 * (r.w + r.h);
    const double d = perim > 0 ? area * unclip_ratio / perim : 0;
    r.w += 2 * d;
    r.h += 2 * d;
    if (std::min(r.w, r.h) < min_size + 2) continue;
    P q[4];
    rect_corners(r, q);
    order_box(q);
    for (int k = 0; k < 4; ++k) {
      boxes[out * 8 + 2 * k] = (float)std::min(std::max(std::round(q[k].x * scale_x), 0.0), (double)src_w);
      boxes[out * 8 + 2 * k + 1] = (float)std::min(std::max(std::round(q[k].y * scale_y), 0.0), (double)src_h);
    }
    out_scores[out] = scores[i];
    ++out;
  }
  return out;
}

// Umeyama similarity transform (no reflection) mapping src[n,2] -> dst[n,2];
// writes the 2x3 forward matrix M (row major).  Used for 5-point face alignment
// (reference: cv2.estimateAffinePartial2D, face onnxrt_backend.py:1382-1417).
void lumen_similarity_transform(const float* src, const float* dst, int n, float* M) {
  double mx = 0, my = 0, ux = 0, uy = 0;
  for (int i = 0; i < n; ++i) { mx += src[2 * i]; my += src[2 * i + 1]; ux += dst[2 * i]; uy += dst[2 * i + 1]; }
  mx /= n; my /= n; ux /= n; uy /= n;
  double sxx = 0, sxy = 0, syx = 0, syy = 0, var = 0;
  for (int i = 0; i < n; ++i) {
    const double ax = src[2 * i] - mx, ay = src[2 * i + 1] - my;
    const double bx = dst[2 * i] - ux, by = dst[2 * i + 1] - uy;
    sxx += bx * ax; sxy += bx * ay; syx += by * ax; syy += by * ay;
    var += ax * ax + ay * ay;
  }
  // for a similarity (rotation + uniform scale) the optimal rotation has
  // a = (sxx + syy), b = (syx - sxy) direction
  const double a = sxx + syy, b = syx - sxy;
  const double norm = std::sqrt(a * a + b * b);
  const double scale = var > 0 ? norm / var : 1.0;
  const double c = norm > 0 ? a / norm : 1.0, s = norm > 0 ? b / norm : 0.0;
  M[0] = (float)(scale * c); M[1] = (float)(-scale * s);
  M[3] = (float)(scale * s); M[4] = (float)(scale * c);
  M[2] = (float)(ux - (M[0] * mx + M[1] * my));
  M[5] = (float)(uy - (M[3] * mx + M[4] * my));
}

int lumen_host_abi_version() { return 1; }

}  // extern "C"
