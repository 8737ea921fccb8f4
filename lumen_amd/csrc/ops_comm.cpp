// torch.ops.lumen.* bindings of the IPC all-reduce (comm.hip): uncached IPC buffer
// allocation, handle export/import, and the collective itself.  Pointers cross the
// Python boundary as int64 (they are process-local device addresses).
#include <ATen/ATen.h>
#include <ATen/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <cstring>
#include <vector>

#include "comm.h"

namespace {

#define CHECK_HIPC(expr)                                                                   \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    TORCH_CHECK(_e == hipSuccess, "lumen HIP error: ", hipGetErrorString(_e), " @ ", #expr); \
  } while (0)

// bytes = control block + 2 parities of `cap` data bytes + 2 parities of `cap` reduced bytes (the
// two-shot form's published sub-slices); zero-filled.
int64_t ar_alloc(int64_t cap) {
  TORCH_CHECK(cap > 0 && cap % 16 == 0, "ar_alloc: capacity must be a positive multiple of 16");
  void* p = nullptr;
  const size_t total = (size_t)lumen::AR_CTL_BYTES + 4 * (size_t)cap;
  CHECK_HIPC(hipExtMallocWithFlags(&p, total, hipDeviceMallocUncached));
  CHECK_HIPC(hipMemset(p, 0, total));
  CHECK_HIPC(hipDeviceSynchronize());
  return reinterpret_cast<int64_t>(p);
}

void ar_free(int64_t ptr) {
  if (ptr) CHECK_HIPC(hipFree(reinterpret_cast<void*>(ptr)));
}

at::Tensor ar_handle(int64_t ptr) {
  hipIpcMemHandle_t h;
  CHECK_HIPC(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr)));
  at::Tensor t = at::empty({(int64_t)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &h, sizeof(h));
  return t;
}

int64_t ar_open(const at::Tensor& handle) {
  hipIpcMemHandle_t h;
  TORCH_CHECK(!handle.is_cuda() && handle.scalar_type() == at::kByte && handle.numel() == (int64_t)sizeof(h),
              "ar_open: cpu uint8 handle of ", sizeof(h), " bytes");
  at::Tensor c = handle.contiguous();
  std::memcpy(&h, c.data_ptr(), sizeof(h));
  void* p = nullptr;
  CHECK_HIPC(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return reinterpret_cast<int64_t>(p);
}

void ar_close(int64_t ptr) {
  if (ptr) CHECK_HIPC(hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr)));
}

int64_t ar_error(int64_t ptr) {
  uint32_t err = 0;
  CHECK_HIPC(hipMemcpy(&err, reinterpret_cast<char*>(ptr) + offsetof(lumen::ArCtl, err), sizeof(err),
                       hipMemcpyDeviceToHost));
  return err;
}

// Enqueue a copy of the error word into out[0] (int32, device) on the current stream: a decode
// graph captures it after its last all-reduce, so the step's result D2H carries the flag and the
// leader can refuse to emit tokens computed from a timed-out (stale) all-reduce.
void ar_error_into(int64_t ptr, at::Tensor out) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kInt && out.numel() >= 1, "ar_error_into: cuda int32 out");
  const at::DeviceGuard g(out.device());
  CHECK_HIPC(hipMemcpyAsync(out.data_ptr(), reinterpret_cast<char*>(ptr) + offsetof(lumen::ArCtl, err), sizeof(uint32_t),
                            hipMemcpyDeviceToDevice, c10::hip::getCurrentHIPStream().stream()));
}

// out = sum over ranks of inp (bf16 or fp32, contiguous, bytes % 16 == 0, bytes <= cap)
void custom_all_reduce(const at::Tensor& inp, at::Tensor out, at::IntArrayRef bases, int64_t rank, int64_t cap,
                       bool two_shot) {
  TORCH_CHECK(inp.is_cuda() && out.is_cuda() && inp.is_contiguous() && out.is_contiguous(), "custom_all_reduce: cuda contiguous");
  TORCH_CHECK(inp.scalar_type() == out.scalar_type() && inp.numel() == out.numel(), "custom_all_reduce: in/out mismatch");
  TORCH_CHECK(inp.scalar_type() == at::kBFloat16 || inp.scalar_type() == at::kFloat, "custom_all_reduce: bf16 or fp32");
  const int64_t world = (int64_t)bases.size();
  TORCH_CHECK(world >= 1 && world <= lumen::AR_MAX_RANKS && rank >= 0 && rank < world, "custom_all_reduce: ranks");
  const int64_t bytes = inp.numel() * inp.element_size();
  TORCH_CHECK(bytes % 16 == 0 && bytes <= cap, "custom_all_reduce: ", bytes, " bytes (cap ", cap, ", multiple of 16)");
  lumen::ArPeers peers{};
  for (int64_t r = 0; r < world; ++r) {
    TORCH_CHECK(bases[r] != 0, "custom_all_reduce: unmapped peer ", r);
    peers.base[r] = reinterpret_cast<char*>(bases[r]);
  }
  const at::DeviceGuard g(inp.device());
  auto fn = two_shot ? lumen::custom_all_reduce_2shot : lumen::custom_all_reduce;
  CHECK_HIPC(fn(inp.data_ptr(), out.data_ptr(), peers, (int)rank, (int)world, bytes,
                inp.scalar_type() == at::kBFloat16 ? 1 : 0, cap, c10::hip::getCurrentHIPStream().stream()));
}

// A HIP stream owned by the caller for the life of the process (never from PyTorch's
// round-robin pool): graph captures key their split-K counters / workspaces by the capture
// stream, so that stream must never be handed to another thread's eager work.
int64_t private_stream(int64_t device) {
  int prev = 0;
  CHECK_HIPC(hipGetDevice(&prev));
  CHECK_HIPC(hipSetDevice((int)device));
  hipStream_t s = nullptr;
  const hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  (void)hipSetDevice(prev);
  CHECK_HIPC(e);
  return reinterpret_cast<int64_t>(s);
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(lumen, m) {
  m.def("private_stream(int device) -> int", &private_stream);
  m.def("ar_alloc(int cap) -> int", &ar_alloc);
  m.def("ar_free(int ptr) -> ()", &ar_free);
  m.def("ar_handle(int ptr) -> Tensor", &ar_handle);
  m.def("ar_open(Tensor handle) -> int", &ar_open);
  m.def("ar_close(int ptr) -> ()", &ar_close);
  m.def("ar_error(int ptr) -> int", &ar_error);
  m.def("custom_all_reduce(Tensor inp, Tensor(o!) out, int[] bases, int rank, int cap, bool two_shot=False) -> ()");
  m.def("ar_error_into(int ptr, Tensor(o!) out) -> ()");
}

TORCH_LIBRARY_IMPL(lumen, CUDA, m) {
  m.impl("custom_all_reduce", &custom_all_reduce);
  m.impl("ar_error_into", &ar_error_into);
}
