// torch.ops.lumen.* registration of the ONNX executor's generic-node kernels (onnx_ops.hip).
#include <ATen/ATen.h>
#include <ATen/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

namespace lumen {
constexpr int EW_DIMS = 6;
struct EwArgs {
  const void* a;
  const void* b;
  void* out;
  int64_t shape[EW_DIMS];
  int64_t sa[EW_DIMS];
  int64_t sb[EW_DIMS];
  int64_t n;
  int op;
  int a_bf16, b_bf16, out_bf16;
};
struct BmmArgs {
  const void* a;
  const void* b;
  float* c;
  int64_t sab, sam, sak, sbb, sbk, sbn, scb, scm, scn;
  int B, M, N, K, a_bf16, b_bf16;
};
hipError_t ew_binary(const EwArgs& a, hipStream_t stream);
hipError_t softmax_rows(const void* x, int x_bf16, void* out, int out_bf16, int64_t rows, int D, hipStream_t stream);
hipError_t resize_bilinear_nhwc(const uint16_t* x, uint16_t* out, int N, int H, int W, int C, int Ho, int Wo, int mode,
                                hipStream_t stream);
hipError_t bmm(const BmmArgs& p, hipStream_t stream);
hipError_t ew_unary(const void* x, int x_bf16, void* out, int out_bf16, int64_t n, int op, float p0, float p1,
                    hipStream_t stream);
}  // namespace lumen

namespace {

#define CHECK_HIP_O(expr)                                                                  \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    TORCH_CHECK(_e == hipSuccess, "lumen HIP error: ", hipGetErrorString(_e), " @ ", #expr); \
  } while (0)

inline hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }

bool fp_ok(const at::Tensor& t) { return t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16; }

// out = a (op) b with numpy broadcasting; out contiguous f32 / bf16 of the broadcast shape
void ew_binary(const at::Tensor& a, const at::Tensor& b, at::Tensor out, int64_t op) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda() && fp_ok(a) && fp_ok(b) && fp_ok(out), "ew_binary: dtypes");
  TORCH_CHECK(out.is_contiguous() && out.dim() <= lumen::EW_DIMS, "ew_binary: out contiguous, <= 6 dims");
  const auto ae = a.expand(out.sizes()), be = b.expand(out.sizes());
  lumen::EwArgs p{};
  const int nd = (int)out.dim(), off = lumen::EW_DIMS - nd;
  for (int d = 0; d < lumen::EW_DIMS; ++d) { p.shape[d] = 1; p.sa[d] = 0; p.sb[d] = 0; }
  for (int d = 0; d < nd; ++d) {
    p.shape[off + d] = out.size(d);
    p.sa[off + d] = ae.stride(d);
    p.sb[off + d] = be.stride(d);
  }
  p.a = a.data_ptr(); p.b = b.data_ptr(); p.out = out.data_ptr(); p.n = out.numel(); p.op = (int)op;
  p.a_bf16 = a.scalar_type() == at::kBFloat16; p.b_bf16 = b.scalar_type() == at::kBFloat16;
  p.out_bf16 = out.scalar_type() == at::kBFloat16;
  const at::DeviceGuard g(a.device());
  CHECK_HIP_O(lumen::ew_binary(p, cur()));
}

void softmax_rows(const at::Tensor& x, at::Tensor out) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && out.is_contiguous() && fp_ok(x) && fp_ok(out) &&
              x.numel() == out.numel() && x.dim() >= 1, "softmax_rows: contiguous f32/bf16");
  const int64_t D = x.size(-1);
  const at::DeviceGuard g(x.device());
  CHECK_HIP_O(lumen::softmax_rows(x.data_ptr(), x.scalar_type() == at::kBFloat16, out.data_ptr(),
                                  out.scalar_type() == at::kBFloat16, x.numel() / std::max<int64_t>(D, 1), (int)D,
                                  cur()));
}

void resize_bilinear_nhwc(const at::Tensor& x, at::Tensor out, int64_t mode) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 4 &&
              x.size(3) % 8 == 0, "resize_bilinear_nhwc: x bf16 NHWC, C % 8 == 0");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.size(0) == x.size(0) &&
              out.size(3) == x.size(3), "resize_bilinear_nhwc: out");
  const at::DeviceGuard g(x.device());
  CHECK_HIP_O(lumen::resize_bilinear_nhwc(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                          reinterpret_cast<uint16_t*>(out.data_ptr()), (int)x.size(0),
                                          (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)out.size(1),
                                          (int)out.size(2), (int)mode, cur()));
}

// c [B, M, N] f32 = a [B, M, K] . b [B, K, N] (any strides)
void bmm(const at::Tensor& a, const at::Tensor& b, at::Tensor c) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && fp_ok(a) && fp_ok(b) && a.dim() == 3 && b.dim() == 3 && c.dim() == 3 &&
              c.scalar_type() == at::kFloat, "bmm: 3-D f32/bf16 operands, f32 out");
  TORCH_CHECK(a.size(0) == b.size(0) && a.size(2) == b.size(1) && c.size(0) == a.size(0) && c.size(1) == a.size(1) &&
              c.size(2) == b.size(2), "bmm: shapes");
  lumen::BmmArgs p{};
  p.a = a.data_ptr(); p.b = b.data_ptr(); p.c = c.data_ptr<float>();
  p.sab = a.stride(0); p.sam = a.stride(1); p.sak = a.stride(2);
  p.sbb = b.stride(0); p.sbk = b.stride(1); p.sbn = b.stride(2);
  p.scb = c.stride(0); p.scm = c.stride(1); p.scn = c.stride(2);
  p.B = (int)a.size(0); p.M = (int)a.size(1); p.K = (int)a.size(2); p.N = (int)b.size(2);
  p.a_bf16 = a.scalar_type() == at::kBFloat16; p.b_bf16 = b.scalar_type() == at::kBFloat16;
  const at::DeviceGuard g(a.device());
  CHECK_HIP_O(lumen::bmm(p, cur()));
}

void ew_unary(const at::Tensor& x, at::Tensor out, int64_t op, double p0, double p1) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && out.is_contiguous() && fp_ok(x) && fp_ok(out) &&
              x.numel() == out.numel(), "ew_unary: contiguous f32/bf16");
  const at::DeviceGuard g(x.device());
  CHECK_HIP_O(lumen::ew_unary(x.data_ptr(), x.scalar_type() == at::kBFloat16, out.data_ptr(),
                              out.scalar_type() == at::kBFloat16, x.numel(), (int)op, (float)p0, (float)p1, cur()));
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(lumen, m) {
  m.def("ew_unary(Tensor x, Tensor(o!) out, int op, float p0, float p1) -> ()");
  m.def("ew_binary(Tensor a, Tensor b, Tensor(o!) out, int op) -> ()");
  m.def("softmax_rows(Tensor x, Tensor(o!) out) -> ()");
  m.def("resize_bilinear_nhwc(Tensor x, Tensor(o!) out, int mode) -> ()");
  m.def("bmm(Tensor a, Tensor b, Tensor(c!) c) -> ()");
}

TORCH_LIBRARY_IMPL(lumen, CUDA, m) {
  m.impl("ew_binary", &ew_binary);
  m.impl("ew_unary", &ew_unary);
  m.impl("softmax_rows", &softmax_rows);
  m.impl("resize_bilinear_nhwc", &resize_bilinear_nhwc);
  m.impl("bmm", &bmm);
}
