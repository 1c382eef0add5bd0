// Microbenchmarks for the partitioned round's local step (c5 shape, one env per 64-lane wave):
//  1. contended counter: lane 0 of every wave takes a record index with atomicAdd (return value
//     used) on one shared counter and stores a 16-byte record there (what emit_req / emit_upd do);
//  2. the same with the index taken from a per-wave fixed slot (no atomic);
//  3. whole-state transfer: every wave loads and stores its env's state (sem 1024 x 8 B, counts
//     256 x 4 B, 128 trains x 24 B), staging the semaphores through 13.9 KB of LDS like k_wave2_part;
//  4. the same with 32-bit semaphore records between launches.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/debug/part_micro scripts/debug/part_micro.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void __launch_bounds__(64) k_atomic(uint32_t* cnt, uint4* out, uint32_t cap, int fixed) {
  __shared__ uint32_t lds[3468];
  const uint32_t e = blockIdx.x;
  lds[threadIdx.x] = e;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t k = fixed ? e : atomicAdd(cnt, 1u);
    if (k < cap) out[k] = make_uint4(e, lds[1], k, 7u);
    uint32_t k2 = fixed ? e + cap / 2 : atomicAdd(cnt + 64, 1u);
    if (k2 < cap) out[k2 + cap] = make_uint4(e, lds[2], k2, 9u);
  }
}

template <bool SEM32>
__global__ void __launch_bounds__(64) k_state(uint64_t* sem, uint32_t* sem32, uint32_t* cnt, uint32_t* tr, uint32_t E) {
  __shared__ uint32_t lds[3468];
  const uint32_t e = blockIdx.x;
  const int l = threadIdx.x;
  uint32_t trv[2][6];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int f = 0; f < 6; ++f) trv[k][f] = tr[((size_t)e * 6 + f) * 128 + k * 64 + l];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const size_t ix = (size_t)e * 1024 + k * 64 + l;
    lds[k * 64 + l] = SEM32 ? sem32[ix] : (uint32_t)sem[ix];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) lds[1024 + k * 64 + l] = cnt[(size_t)e * 256 + k * 64 + l];
  __syncthreads();
  // a little work on the state
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int f = 0; f < 6; ++f) trv[k][f] += lds[(l * 7 + f) & 1023];
  lds[(l * 13) & 1023] += 1;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int f = 0; f < 6; ++f) tr[((size_t)e * 6 + f) * 128 + k * 64 + l] = trv[k][f];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const size_t ix = (size_t)e * 1024 + k * 64 + l;
    if (SEM32) sem32[ix] = lds[k * 64 + l];
    else sem[ix] = lds[k * 64 + l] | ((uint64_t)1 << 40);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) cnt[(size_t)e * 256 + k * 64 + l] = lds[1024 + k * 64 + l];
}

int main() {
  const uint32_t E = 16384;
  uint32_t* cnt;
  uint4* out;
  CK(hipMalloc(&cnt, 1024));
  CK(hipMalloc(&out, (size_t)4 * E * 16));
  uint64_t* sem;
  uint32_t *sem32, *cnts, *tr;
  CK(hipMalloc(&sem, (size_t)E * 1024 * 8));
  CK(hipMalloc(&sem32, (size_t)E * 1024 * 4));
  CK(hipMalloc(&cnts, (size_t)E * 256 * 4));
  CK(hipMalloc(&tr, (size_t)E * 128 * 6 * 4));
  CK(hipMemset(sem, 0, (size_t)E * 1024 * 8));
  CK(hipMemset(sem32, 0, (size_t)E * 1024 * 4));
  CK(hipMemset(cnts, 0, (size_t)E * 256 * 4));
  CK(hipMemset(tr, 0, (size_t)E * 128 * 6 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int mode = 0; mode < 4; ++mode) {
    float best = 1e9f;
    for (int it = 0; it < 20; ++it) {
      CK(hipMemset(cnt, 0, 1024));
      CK(hipEventRecord(a));
      if (mode == 0) k_atomic<<<E, 64>>>(cnt, out, 2 * E, 0);
      else if (mode == 1) k_atomic<<<E, 64>>>(cnt, out, 2 * E, 1);
      else if (mode == 2) k_state<false><<<E, 64>>>(sem, sem32, cnts, tr, E);
      else k_state<true><<<E, 64>>>(sem, sem32, cnts, tr, E);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (it > 2 && ms < best) best = ms;
    }
    const char* names[4] = {"2 contended atomicAdd-return + record per wave", "2 fixed-slot records per wave",
                            "state load+store, 64-bit sem", "state load+store, 32-bit sem"};
    printf("%-50s %8.1f us  (%u waves, 64-thread blocks, 13.9 KB LDS)\n", names[mode], best * 1e3, E);
  }
  return 0;
}
