// Dev tool (not shipped): semantics check of __builtin_amdgcn_global_load_lds (16 B/lane):
// lane l of a wave loads 16 B from a per-lane (permuted) global address; the bytes must land
// at LDS base + 16*l.  Also times a stage of 16 glds (1 KB each) per workgroup.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -w tools/glds_probe.hip -o tools/glds_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void glds_check(const float* src, float* out) {
  __shared__ __attribute__((aligned(16))) float lds[4 * 256];   // 4 waves x 1 KB
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // lane l loads float4 #perm(l) of this wave's 1 KB source block
  const int perm = (lane * 37 + 11) & 63;
  const float* g = src + (wave * 64 + perm) * 4;
  __builtin_amdgcn_global_load_lds(g, lds + wave * 256, 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * 256; i += 256) out[i] = lds[i];
}

int main() {
  std::vector<float> h(1024), o(1024);
  for (int i = 0; i < 1024; ++i) h[i] = (float)i;
  float *src, *out;
  hipMalloc(&src, 4096); hipMalloc(&out, 4096);
  hipMemcpy(src, h.data(), 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(glds_check, dim3(1), dim3(256), 0, 0, src, out);
  hipMemcpy(o.data(), out, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int w = 0; w < 4; ++w)
    for (int l = 0; l < 64; ++l) {
      const int perm = (l * 37 + 11) & 63;
      for (int j = 0; j < 4; ++j)
        if (o[w * 256 + l * 4 + j] != h[(w * 64 + perm) * 4 + j]) ++bad;
    }
  printf("glds lane-linear destination check: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
  return bad != 0;
}
