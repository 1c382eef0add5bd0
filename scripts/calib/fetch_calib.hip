// FETCH_SIZE / WRITE_SIZE calibration for the bench kernel's access shapes (round-4 verdict item 7).
//
// MI355X_MICROARCH.md § HBM calibrates FETCH_SIZE only for 16-B-per-lane coalesced streaming reads
// (reported = 1/2 of the bytes).  The c3 kernel's HBM accesses are scattered: 4-B (switch, train) slot
// words, 8-B Q cells, 32-B compact Q rows (<= 4 doubles), 4-B key-set atomics, 16-B move-table rows.  Each
// kernel below performs exactly one access of one shape per lane, every lane on its own 128-B line of a
// 1 GiB table (a bijection of the line index: no line is touched twice inside a launch, and the table is
// 4x the 256-MiB Infinity Cache), so the bytes the lanes ask for -- and the lines they touch -- are known
// exactly.  rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE per kernel then gives the counter's bytes per request
// for each shape (scripts/calib/fetch_calib.py turns them into the factors scripts/pmc_summary.py uses).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/calib/fetch_calib.bin scripts/calib/fetch_calib.hip
// Run:   scripts/calib/fetch_calib.bin   (prints one JSON line: the launches and their known byte counts)
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

constexpr uint64_t kTableBytes = 1ull << 30;           // 1 GiB
constexpr uint64_t kLines = kTableBytes / 128;         // 2^23 lines of 128 B
constexpr uint64_t kN = 1ull << 22;                    // accesses per launch (half the lines)
constexpr uint32_t kMult = 0x9E3779B1u;                // odd: i -> i * kMult mod 2^23 is a bijection

__device__ __forceinline__ uint64_t line_of(uint64_t i, uint32_t salt) { return (i * kMult + salt) & (kLines - 1); }
__device__ __forceinline__ uint32_t mix(uint64_t i) {
  uint32_t x = (uint32_t)i * 0x85EBCA6Bu;
  x ^= x >> 13;
  return x * 0xC2B2AE35u;
}

// one W-byte read per lane, at a W-aligned offset of its own line
template <int W>
__global__ void __launch_bounds__(256) k_rd(const uint8_t* __restrict__ tab, uint32_t salt, uint32_t* __restrict__ sink) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kN) return;
  const uint32_t off = (mix(i) % (128 / W)) * W;
  const uint8_t* p = tab + line_of(i, salt) * 128 + off;
  uint32_t acc = 0;
  if constexpr (W == 4) {
    acc = *(const uint32_t*)p;
  } else if constexpr (W == 8) {
    const uint2 v = *(const uint2*)p;
    acc = v.x ^ v.y;
  } else {
#pragma unroll
    for (int k = 0; k < W / 16; ++k) {
      const uint4 v = ((const uint4*)p)[k];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x9E3779B9u) sink[i & 1023] = acc;  // (practically never: keeps the loads)
}

// four separate f64 loads of a 32-B row (the bench kernel's compact Q row as the compiler may issue it)
__global__ void __launch_bounds__(256) k_rd_row4(const uint8_t* __restrict__ tab, uint32_t salt, uint32_t* __restrict__ sink) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kN) return;
  const double* p = (const double*)(tab + line_of(i, salt) * 128 + (mix(i) % 4) * 32);
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) s += p[k];
  if (s == 1.2345) sink[i & 1023] = 1u;
}

// one W-byte store per lane
template <int W>
__global__ void __launch_bounds__(256) k_wr(uint8_t* __restrict__ tab, uint32_t salt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kN) return;
  const uint32_t off = (mix(i) % (128 / W)) * W;
  uint8_t* p = tab + line_of(i, salt) * 128 + off;
  if constexpr (W == 4) {
    *(uint32_t*)p = (uint32_t)i;
  } else if constexpr (W == 8) {
    *(double*)p = (double)i;
  } else {
#pragma unroll
    for (int k = 0; k < W / 16; ++k) ((uint4*)p)[k] = make_uint4((uint32_t)i, k, 1, 2);
  }
}

// one 4-B atomicOr per lane (the key-set insert)
__global__ void __launch_bounds__(256) k_atom_or(uint8_t* __restrict__ tab, uint32_t salt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kN) return;
  uint32_t* p = (uint32_t*)(tab + line_of(i, salt) * 128 + (mix(i) % 32) * 4);
  atomicOr(p, 1u << (i & 31));
}

// the guide's calibrated case: 16 B per lane, coalesced, over kStream bytes
constexpr uint64_t kStream = 512ull << 20;
__global__ void __launch_bounds__(256) k_stream16(const uint4* __restrict__ src, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < kStream / 16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[threadIdx.x] = acc;
}

int main() {
  uint8_t* tab = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&tab, kTableBytes));
  CK(hipMalloc(&sink, 4096 * 4));
  CK(hipMemset(tab, 1, kTableBytes));
  CK(hipDeviceSynchronize());
  const unsigned blocks = (unsigned)(kN / 256);
  const int reps = 3;
  printf("{\"table_bytes\": %llu, \"accesses_per_launch\": %llu, \"launches_per_kernel\": %d, \"kernels\": {", (unsigned long long)kTableBytes,
         (unsigned long long)kN, reps);
  bool first = true;
  auto rec = [&](const char* name, uint64_t bytes_per_access, uint64_t lines) {
    printf("%s\"%s\": {\"bytes\": %llu, \"lines\": %llu}", first ? "" : ", ", name, (unsigned long long)(bytes_per_access * kN),
           (unsigned long long)lines);
    first = false;
  };
  for (int r = 0; r < reps; ++r) {
    const uint32_t salt = 0x1234567u * (r + 1);
    k_rd<4><<<blocks, 256>>>(tab, salt, sink);
    k_rd<8><<<blocks, 256>>>(tab, salt + 1, sink);
    k_rd<16><<<blocks, 256>>>(tab, salt + 2, sink);
    k_rd<32><<<blocks, 256>>>(tab, salt + 3, sink);
    k_rd_row4<<<blocks, 256>>>(tab, salt + 4, sink);
    k_rd<64><<<blocks, 256>>>(tab, salt + 5, sink);
    k_rd<128><<<blocks, 256>>>(tab, salt + 6, sink);
    k_wr<4><<<blocks, 256>>>(tab, salt + 7);
    k_wr<8><<<blocks, 256>>>(tab, salt + 8);
    k_wr<32><<<blocks, 256>>>(tab, salt + 9);
    k_wr<128><<<blocks, 256>>>(tab, salt + 10);
    k_atom_or<<<blocks, 256>>>(tab, salt + 11);
    k_stream16<<<4096, 256>>>((const uint4*)(tab + (r & 1) * kStream), sink);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  rec("k_rd<4>", 4, kN);
  rec("k_rd<8>", 8, kN);
  rec("k_rd<16>", 16, kN);
  rec("k_rd<32>", 32, kN);
  rec("k_rd_row4", 32, kN);
  rec("k_rd<64>", 64, kN);
  rec("k_rd<128>", 128, kN);
  rec("k_wr<4>", 4, kN);
  rec("k_wr<8>", 8, kN);
  rec("k_wr<32>", 32, kN);
  rec("k_wr<128>", 128, kN);
  rec("k_atom_or", 4, kN);
  printf(", \"k_stream16\": {\"bytes\": %llu, \"lines\": %llu}}}\n", (unsigned long long)kStream, (unsigned long long)(kStream / 128));
  CK(hipFree(tab));
  CK(hipFree(sink));
  return 0;
}
