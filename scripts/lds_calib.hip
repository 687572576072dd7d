// lds_calib.hip — calibration of the gfx950 LDS counters: which of
// SQ_LDS_BANK_CONFLICT / SQ_LDS_ADDR_CONFLICT measures bank conflicts, against access patterns
// whose conflict cycles are known from the bank rule (MI355X_MICROARCH.md §LDS: ds_read_b32 serves
// lanes {0-31} and {32-63} in one LDS cycle each when conflict-free, bank = (a/4) mod 32; N
// distinct addresses on one bank within a group cost N cycles).
//
// One kernel per pattern (rocprofv3 reports each dispatch on its own row); every thread issues
// kReads ds_read_b32 of its pattern's address, 256-thread workgroups, one per CU-slot of the grid.
// Expected LDS-array cycles per wave-instruction (IDX_ACTIVE) and extra conflict cycles (BANK):
//   stride1     lane l reads word l               2 cycles, 0 extra
//   stride2     word 2l  (2 lanes per bank)        4 cycles, 2 extra
//   stride32    word 32l (32 lanes on bank 0)     64 cycles, 62 extra
//   bcast       word 0 for every lane              2 cycles, 0 extra (broadcast)
//   stride33    word 33l (one lane per bank)       2 cycles, 0 extra
//   w_stride32  ds_write_b32 word 32l              LDS array 64 cycles, 62 extra
// Build: make lds_calib (hipcc --offload-arch=gfx950); run: scripts/lds_calib.sh on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kThreads = 256;
constexpr int kReads = 4096;

template <int STRIDE, bool WRITE>
__global__ void __launch_bounds__(kThreads) lds_pattern(uint32_t* out, uint32_t salt) {
  __shared__ uint32_t s[64 * 33 + 64];
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t i = threadIdx.x; i < sizeof(s) / 4; i += kThreads) s[i] = i ^ salt;
  __syncthreads();
  const uint32_t w = STRIDE < 0 ? 0u : lane * (uint32_t)STRIDE;  // STRIDE < 0: broadcast
  uint32_t acc = 0;
  // explicit ds_read_b32 / ds_write_b32 (a volatile C++ access through a generic pointer would be a
  // flat load); LDS byte address of the pattern's word
  const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)&s[w];
  for (int k = 0; k < kReads; ++k) {
    if (WRITE) {
      asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(addr), "v"((uint32_t)k) : "memory");
      acc += 1u;
    } else {
      uint32_t x;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(addr) : "memory");
      acc += x;
    }
  }
  if (acc == 0xdeadbeefu) out[blockIdx.x * kThreads + threadIdx.x] = acc;
}

template <class K>
static void run(const char* name, K kern, uint32_t* d, int grid) {
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, 0, d, 1u);
  if (hipDeviceSynchronize() != hipSuccess) {
    fprintf(stderr, "%s failed\n", name);
    exit(1);
  }
  printf("%s done: %d workgroups x %d threads x %d accesses\n", name, grid, kThreads, kReads);
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = ncu > 0 ? ncu : 256;
  uint32_t* d = nullptr;
  if (hipMalloc(&d, (size_t)grid * kThreads * 4) != hipSuccess) return 1;
  run("stride1", lds_pattern<1, false>, d, grid);
  run("stride2", lds_pattern<2, false>, d, grid);
  run("stride32", lds_pattern<32, false>, d, grid);
  run("bcast", lds_pattern<-1, false>, d, grid);
  run("stride33", lds_pattern<33, false>, d, grid);
  run("w_stride32", lds_pattern<32, true>, d, grid);
  (void)hipFree(d);
  return 0;
}
