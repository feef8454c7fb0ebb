// launch_floor.hip: what a kernel that stands down costs on one stream (r06;
// VERDICT r05 item 2, the gated fallback behind every speculative batch).
// Each case enqueues `iters` launches back to back and syncs once; the figure
// is the stream's wall time per launch. The "chain" cases put the launches
// behind a ~100 us work kernel, as the fallback sits behind a select, and
// report the added time per stand-down.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_floor tools/launch_floor.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <functional>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void empty_k() {}

__global__ __launch_bounds__(256) void gated_small(const uint32_t* run_if, float* out) {
  if (*run_if == 0u) return;
  out[blockIdx.x * 256 + threadIdx.x] = 1.f;
}

// the shape of the fallback's launches: 512 threads, most of the LDS
__global__ __launch_bounds__(512) void gated_big(const uint32_t* run_if, float* out) {
  __shared__ float lds[36 * 1024];
  if (*run_if == 0u) return;
  lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  out[blockIdx.x * 512 + threadIdx.x] = lds[511 - threadIdx.x];
}

// ~busy_iters dependent FMAs per lane on every CU: a stand-in for the select
__global__ __launch_bounds__(256) void work_k(float* out, int busy_iters) {
  float a = (float)threadIdx.x, b = 1.0001f;
  for (int i = 0; i < busy_iters; ++i) a = fmaf(a, b, 0.5f);
  out[blockIdx.x * 256 + threadIdx.x] = a;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint32_t* flag;
  float* out;
  CK(hipMalloc(&flag, 64));
  CK(hipMemset(flag, 0, 64));
  CK(hipMalloc(&out, 64 << 20));
  const int iters = 4000;
  auto per_launch = [&](const std::function<void()>& f, int n) -> double {
    for (int i = 0; i < 50; ++i) f();
    (void)hipStreamSynchronize(st);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) f();
    (void)hipStreamSynchronize(st);
    const auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
  };
  std::printf("{\"tool\": \"launch_floor\", \"us_per_launch\": {");
  struct C {
    const char* name;
    std::function<void()> f;
  };
  std::vector<C> cases = {
      {"empty_1x64", [&] { hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, st); }},
      {"gated_1x256", [&] { hipLaunchKernelGGL(gated_small, dim3(1), dim3(256), 0, st, flag, out); }},
      {"gated_256x256",
       [&] { hipLaunchKernelGGL(gated_small, dim3(256), dim3(256), 0, st, flag, out); }},
      {"gated_1024x256",
       [&] { hipLaunchKernelGGL(gated_small, dim3(1024), dim3(256), 0, st, flag, out); }},
      {"gated_big_256x512",
       [&] { hipLaunchKernelGGL(gated_big, dim3(256), dim3(512), 0, st, flag, out); }},
  };
  bool first = true;
  for (auto& c : cases) {
    std::printf("%s\"%s\": %.3f", first ? "" : ", ", c.name, per_launch(c.f, iters));
    first = false;
    std::fflush(stdout);
  }
  // work kernel alone, then followed by 1 / 4 stand-downs of the big shape
  const int busy = 20000;
  auto work = [&] { hipLaunchKernelGGL(work_k, dim3(1024), dim3(256), 0, st, out, busy); };
  const double w0 = per_launch(work, 500);
  std::printf(", \"work\": %.3f", w0);
  for (int nd : {1, 4}) {
    const double w = per_launch(
        [&] {
          work();
          for (int j = 0; j < nd; ++j)
            hipLaunchKernelGGL(gated_big, dim3(256), dim3(512), 0, st, flag, out);
        },
        500);
    std::printf(", \"work+%d_standdown_added_per_launch\": %.3f", nd, (w - w0) / nd);
  }
  for (int nd : {1, 4}) {
    const double w = per_launch(
        [&] {
          work();
          for (int j = 0; j < nd; ++j)
            hipLaunchKernelGGL(gated_small, dim3(1), dim3(256), 0, st, flag, out);
        },
        500);
    std::printf(", \"work+%d_tiny_added_per_launch\": %.3f", nd, (w - w0) / nd);
  }
  std::printf("}}\n");
  CK(hipGetLastError());
  return 0;
}
