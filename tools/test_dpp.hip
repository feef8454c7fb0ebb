// Unit check of wave_sum_dpp against wave_sum on the device (debug aid).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/test_dpp.hip -o tools/test_dpp
#include "../gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd/csrc/vs_kernels.hip"
#include <cstdio>
#include <vector>
using namespace vsk;
__global__ void probe(const float* in, float* out) {
  const int lane = threadIdx.x & 63;
  const float v = in[blockIdx.x * 64 + lane];
  float s = v;
  s += dpp_f<0xB1>(s);
  out[(blockIdx.x * 8 + 0) * 64 + lane] = s;
  s += dpp_f<0x4E>(s);
  out[(blockIdx.x * 8 + 1) * 64 + lane] = s;
  s += dpp_f<0x141>(s);
  out[(blockIdx.x * 8 + 2) * 64 + lane] = s;
  s += dpp_f<0x140>(s);
  out[(blockIdx.x * 8 + 3) * 64 + lane] = s;
  out[(blockIdx.x * 8 + 4) * 64 + lane] = wave_sum_dpp(v);
  out[(blockIdx.x * 8 + 5) * 64 + lane] = wave_sum(v);
}
int main() {
  const int nb = 4;
  std::vector<float> h(nb * 64), o(nb * 8 * 64);
  for (int i = 0; i < nb * 64; ++i) h[i] = (float)(i % 64) + (i / 64) * 1000.f;
  float *din, *dout;
  hipMalloc(&din, h.size() * 4);
  hipMalloc(&dout, o.size() * 4);
  hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, 0, din, dout);
  hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
  const char* names[6] = {"xor1", "xor2", "halfmirror", "mirror", "dpp_sum", "ref_sum"};
  for (int st = 0; st < 6; ++st) {
    printf("%-10s:", names[st]);
    for (int l = 0; l < 64; l += 1) printf(" %g", o[(0 * 8 + st) * 64 + l]);
    printf("\n");
  }
  return 0;
}
