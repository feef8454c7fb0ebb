// rt_floor.hip: where a small host-API search's fixed cost goes. The
// one-launch small path did not move the ~37 us per
// call, so this times the pieces of vs_search's round trip alone, on one
// stream, host clock, p50 over 20000 calls each:
//   launch   one empty kernel + event record + polled wait
//   h2d      3 KiB pinned -> device copy + event + wait
//   d2h      40 B device -> pinned copy + event + wait
//   full     h2d + kernel + d2h + event + wait (vs_search's shape)
//   full_sync  the same, hipStreamSynchronize instead of the polled event
//   out_map  h2d + kernel writing its 40 B to mapped pinned memory + event
//   in_map   kernel reading its 3 KiB from mapped pinned memory + d2h + event
//   graph    full's three operations captured once into a hipGraph, one
//            graph launch + event + wait per call (r03)
//   flag_map h2d + a kernel that writes its keys and then a sequence word to
//            mapped pinned memory (system-scope fence between); the host
//            spins on the word, no event (r03)
//   arg_flag the query passed by value in the kernel arguments (3 KiB, no
//            H2D copy) + flag_map's completion word (r03)
//   vs_search  the engine's host API on config C1 (221 x 768 fp32 cosine,
//            one query, k = 5): everything above plus the engine's own work
//
//   hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/rt_floor tools/rt_floor.hip \
//     -L<pkg>/lib -lvsearch -Wl,-rpath,<pkg>/lib
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#include "vsearch.h"

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void touch(const float* __restrict__ in, uint64_t* __restrict__ out, int n) {
  // one workgroup: sum the query (a dependent read of every element) and
  // write 5 keys, like the small path's first and last accesses
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += in[i];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < 256; ++i) t += red[i];
    for (int i = 0; i < 5; ++i) out[i] = (uint64_t)__float_as_uint(t) + (uint64_t)i;
  }
}

// keys to mapped host memory, then (after a system-scope fence) the call's
// sequence number: a host that sees the number sees the keys
__global__ void touch_flag(const float* __restrict__ in, uint64_t* out, int n, uint64_t seq) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += in[i];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < 256; ++i) t += red[i];
    for (int i = 0; i < 5; ++i) out[i] = (uint64_t)__float_as_uint(t) + (uint64_t)i;
    __threadfence_system();
    __hip_atomic_store(out + 7, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// the query travels in the kernel's argument segment (read through the
// segment pointer, vector loads: the struct is the first argument)
struct QArg {
  float v[768];
};
__global__ void touch_arg(QArg qa, uint64_t* out, int n, uint64_t seq) {
  const __attribute__((address_space(4))) float* in =
      (const __attribute__((address_space(4))) float*)__builtin_amdgcn_kernarg_segment_ptr();
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += in[i];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < 256; ++i) t += red[i];
    for (int i = 0; i < 5; ++i) out[i] = (uint64_t)__float_as_uint(t) + (uint64_t)i;
    __threadfence_system();
    __hip_atomic_store(out + 7, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static void wait_polled(hipEvent_t ev) {
  while (hipEventQuery(ev) == hipErrorNotReady) {
  }
}

static double p50(std::vector<double>& v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const int n = 768, iters = 20000;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  float *h_in, *d_in, *m_in;
  uint64_t *h_out, *d_out, *m_out;
  CK(hipHostMalloc(&h_in, n * 4, hipHostMallocDefault));
  CK(hipHostMalloc(&h_out, 64, hipHostMallocDefault));
  CK(hipHostMalloc(&m_in, n * 4, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc(&m_out, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipMalloc(&d_in, n * 4));
  CK(hipMalloc(&d_out, 64));
  for (int i = 0; i < n; ++i) h_in[i] = m_in[i] = 1.0f / (float)(i + 1);

  struct Case {
    const char* name;
    std::function<void()> body;
    int sync;  // 0: event + polled wait, 1: hipStreamSynchronize, 2: the body waits
  };
  hipGraph_t graph;
  hipGraphExec_t gexec;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  (void)hipMemcpyAsync(d_in, h_in, n * 4, hipMemcpyHostToDevice, st);
  hipLaunchKernelGGL(touch, dim3(1), dim3(256), 0, st, d_in, d_out, n);
  (void)hipMemcpyAsync(h_out, d_out, 40, hipMemcpyDeviceToHost, st);
  CK(hipStreamEndCapture(st, &graph));
  CK(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
  uint64_t seq = 0;
  std::vector<Case> cases = {
      {"launch", [&] { hipLaunchKernelGGL(touch, dim3(1), dim3(256), 0, st, d_in, d_out, n); }, 0},
      {"h2d", [&] { (void)hipMemcpyAsync(d_in, h_in, n * 4, hipMemcpyHostToDevice, st); }, 0},
      {"d2h", [&] { (void)hipMemcpyAsync(h_out, d_out, 40, hipMemcpyDeviceToHost, st); }, 0},
      {"full",
       [&] {
         (void)hipMemcpyAsync(d_in, h_in, n * 4, hipMemcpyHostToDevice, st);
         hipLaunchKernelGGL(touch, dim3(1), dim3(256), 0, st, d_in, d_out, n);
         (void)hipMemcpyAsync(h_out, d_out, 40, hipMemcpyDeviceToHost, st);
       },
       0},
      {"full_sync",
       [&] {
         (void)hipMemcpyAsync(d_in, h_in, n * 4, hipMemcpyHostToDevice, st);
         hipLaunchKernelGGL(touch, dim3(1), dim3(256), 0, st, d_in, d_out, n);
         (void)hipMemcpyAsync(h_out, d_out, 40, hipMemcpyDeviceToHost, st);
       },
       1},
      {"out_map",
       [&] {
         (void)hipMemcpyAsync(d_in, h_in, n * 4, hipMemcpyHostToDevice, st);
         hipLaunchKernelGGL(touch, dim3(1), dim3(256), 0, st, d_in, m_out, n);
       },
       0},
      {"in_map",
       [&] {
         hipLaunchKernelGGL(touch, dim3(1), dim3(256), 0, st, m_in, d_out, n);
         (void)hipMemcpyAsync(h_out, d_out, 40, hipMemcpyDeviceToHost, st);
       },
       0},
      {"arg_flag",
       [&] {
         ++seq;
         QArg qa;
         std::memcpy(qa.v, h_in, sizeof(qa.v));
         hipLaunchKernelGGL(touch_arg, dim3(1), dim3(256), 0, st, qa, m_out, n, seq);
         while (__atomic_load_n((volatile uint64_t*)(m_out + 7), __ATOMIC_ACQUIRE) != seq) {
         }
       },
       2},
      {"graph", [&] { (void)hipGraphLaunch(gexec, st); }, 0},
      {"flag_map",
       [&] {
         ++seq;
         (void)hipMemcpyAsync(d_in, h_in, n * 4, hipMemcpyHostToDevice, st);
         hipLaunchKernelGGL(touch_flag, dim3(1), dim3(256), 0, st, d_in, m_out, n, seq);
         while (__atomic_load_n((volatile uint64_t*)(m_out + 7), __ATOMIC_ACQUIRE) != seq) {
         }
       },
       2},
  };
  std::printf("{\"tool\": \"rt_floor\", \"p50_us\": {");
  bool first = true;
  for (auto& c : cases) {
    std::vector<double> t;
    t.reserve(iters);
    for (int i = 0; i < iters + 500; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      c.body();
      if (c.sync == 1) {
        CK(hipStreamSynchronize(st));
      } else if (c.sync == 0) {
        CK(hipEventRecord(ev, st));
        wait_polled(ev);
      }
      const auto t1 = std::chrono::steady_clock::now();
      if (i >= 500) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::printf("%s\"%s\": %.2f", first ? "" : ", ", c.name, p50(t));
    first = false;
    std::fflush(stdout);
  }
  {
    vs_engine* eng = nullptr;
    vs_config cfg = {0, 0u};
    if (vs_open(&cfg, &eng) != VS_OK || vs_collection_create(eng, "c1", n, 0, 0, 0, 0) != VS_OK ||
        vs_generate(eng, "c1", 221, 7) != VS_OK) {
      std::fprintf(stderr, "engine: %s\n", vs_last_error());
      return 1;
    }
    float sc[5];
    uint64_t rw[5];
    uint32_t cnt;
    std::vector<double> t;
    for (int i = 0; i < iters + 500; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      if (vs_search(eng, "c1", h_in, 1, n, 5, sc, rw, &cnt) != VS_OK) return 1;
      const auto t1 = std::chrono::steady_clock::now();
      if (i >= 500) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::printf(", \"vs_search\": %.2f", p50(t));
    vs_close(eng);
  }
  std::printf("}}\n");
  CK(hipGetLastError());
  return 0;
}
