// lds_occ.hip — how many 256-thread workgroups a gfx950 CU holds at once for a given dynamic LDS
// size (the tile planner's per_cu() assumes floor(160 KiB / bytes); r05 found layouts where the
// hardware held one fewer). Each workgroup records its start (s_memrealtime, 100 MHz) and spins for
// ~40 us; the workgroups that started within 10 us of the first were resident together.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/lds_occ.hip -o scripts/lds_occ
// Run (GPU box): scripts/lds_occ [lo] [hi] [step]  — one line per LDS size.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void __launch_bounds__(256) probe(unsigned long long* start, unsigned* sink) {
  extern __shared__ unsigned lds[];
  if (threadIdx.x == 0) start[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned v = lds[(threadIdx.x * 7) & 255];
  while (__builtin_amdgcn_s_memrealtime() - t0 < 4000) v = v * 1664525u + 1013904223u;
  if (v == 0x12345678u) sink[threadIdx.x] = v;  // keeps the loop
}

int main(int argc, char** argv) {
  const int lo = argc > 1 ? atoi(argv[1]) : 32768, hi = argc > 2 ? atoi(argv[2]) : 82944,
            step = argc > 3 ? atoi(argv[3]) : 512;
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const int grid = ncu * 8;
  unsigned long long* d_start = nullptr;
  unsigned* d_sink = nullptr;
  hipMalloc(&d_start, grid * sizeof(unsigned long long));
  hipMalloc(&d_sink, 256 * sizeof(unsigned));
  std::vector<unsigned long long> st(grid);
  int prev = -1;
  for (int b = lo; b <= hi; b += step) {
    int occ = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)probe, 256, b);
    hipLaunchKernelGGL(probe, dim3(grid), dim3(256), b, 0, d_start, d_sink);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("lds %d: launch failed\n", b);
      return 1;
    }
    hipMemcpy(st.data(), d_start, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    const unsigned long long first = *std::min_element(st.begin(), st.end());
    int together = 0;
    for (unsigned long long x : st) together += x <= first + 1000;
    const int per_cu = together / ncu;
    if (per_cu != prev || b + step > hi)
      printf("lds %6d B: %5d workgroups resident together = %.2f per CU (floor(160 KiB / lds) = %d, occupancy API %d)\n", b,
             together, (double)together / ncu, (160 * 1024) / b, occ);
    prev = per_cu;
  }
  hipFree(d_start);
  hipFree(d_sink);
  return 0;
}
