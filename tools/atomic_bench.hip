// Micro-benchmark (not part of the product): throughput of agent-scope
// atomic adds from one lane per workgroup, 256 workgroups, on 1 / 8 / 64
// counters (counter = blockIdx % C, each on its own 256-B line).
//   hipcc --offload-arch=gfx950 -O3 tools/atomic_bench.hip -o tools/atomic_bench
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* c, int stride_words, int ncnt, int iters, unsigned* sink) {
  if (threadIdx.x != 0) return;
  unsigned* p = c + (blockIdx.x % ncnt) * stride_words;
  unsigned acc = 0;
  for (int i = 0; i < iters; ++i)
    acc += __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  sink[blockIdx.x] = acc;
}

int main() {
  unsigned *c, *sink;
  hipMalloc(&c, 64 * 256 * 4);
  hipMalloc(&sink, 4096 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 200;
  for (int ncnt : {1, 8, 64}) {
    for (int nwg : {1, 8, 256}) {
      float best = 1e9;
      for (int r = 0; r < 5; ++r) {
        hipMemset(c, 0, 64 * 256 * 4);
        hipEventRecord(a, 0);
        hipLaunchKernelGGL(k, dim3(nwg), dim3(64), 0, 0, c, 64, ncnt, iters, sink);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
      }
      printf("counters %2d  workgroups %3d: %.1f us total, %.3f us per atomic per wg, %.1f M atomics/s\n",
             ncnt, nwg, best * 1e3, best * 1e3 / iters, (double)nwg * iters / best / 1e3);
    }
  }
  return 0;
}
