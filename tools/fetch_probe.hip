// fetch_probe.hip — how FETCH_SIZE counts a kernel's HBM reads on gfx950 for
// the access patterns of the bounce-level engine.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_probe tools/fetch_probe.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d OUT -o fp --output-format csv -- tools/fetch_probe
//
// Every kernel reads a known number of bytes exactly once from a 2 GiB arena
// (no reuse, larger than the L2 and MALL), then writes one word per block:
//   k_stream      16-B vector loads, consecutive lanes consecutive (the
//                 pattern MI355X_MICROARCH.md's x2 correction is stated for)
//   k_scatter<R>  one R-byte record per lane (R / 16 loads of 16 B), records
//                 at a pseudo-random permutation of the arena's record slots
//                 (the tree records of k_tree_finalize: R = 32; the staged ray
//                 records of k_level_c: R = 80)
//   k_runs<R>     the same records in runs of 64 consecutive ones per wave,
//                 runs in permuted order (a level queue's chunk)
// The program prints each kernel's algorithmic bytes; tools/pmc_json.py
// divides the counted FETCH_SIZE by them (fetch_factor per pattern).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                      \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr size_t ARENA = (size_t)2 << 30;

__global__ void k_stream(const float4* __restrict__ a, size_t n, float* out) {
  float acc = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678f) out[blockIdx.x] = acc;   // never true for the zeroed arena: no store traffic
}

// slot i of a permutation of [0, n) (n a power of two): an odd multiplier and
// an xor-shift, both bijections mod n
__device__ __forceinline__ size_t perm(size_t i, size_t n) {
  size_t x = (i * 0x9E3779B97F4A7C15ull) & (n - 1);
  x ^= x >> 7;
  return (x * 0xBF58476D1CE4E5B9ull) & (n - 1);
}

template <int R>
__global__ void k_scatter(const char* __restrict__ a, size_t nrec, float* out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= nrec) return;
  const float4* r = reinterpret_cast<const float4*>(a + perm(i, nrec) * R);
  float acc = 0.0f;
#pragma unroll
  for (int k = 0; k < R / 16; k++) {
    const float4 v = r[k];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678f) out[blockIdx.x] = acc;
}

template <int R>
__global__ void k_runs(const char* __restrict__ a, size_t nrec, float* out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= nrec) return;
  const size_t run = perm(i >> 6, nrec >> 6);
  const float4* r = reinterpret_cast<const float4*>(a + ((run << 6) + (i & 63)) * R);
  float acc = 0.0f;
#pragma unroll
  for (int k = 0; k < R / 16; k++) {
    const float4 v = r[k];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678f) out[blockIdx.x] = acc;
}

int main() {
  char* a;
  float* out;
  CHK(hipMalloc(&a, ARENA));
  CHK(hipMemset(a, 0, ARENA));
  CHK(hipMalloc(&out, 1 << 20));
  CHK(hipDeviceSynchronize());
  // 16 MiB flush between kernels: nothing of one kernel's reads stays in L2/MALL for the next
  const size_t n16 = ARENA / 16;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const float4*>(a), n16, out);
    CHK(hipDeviceSynchronize());
    printf("k_stream bytes %zu\n", ARENA);
    {
      const size_t nrec = ((size_t)1 << 26);     // 64 Mi records of 32 B = 2 GiB
      hipLaunchKernelGGL(k_scatter<32>, dim3((unsigned)(nrec / 256)), dim3(256), 0, 0, a, nrec, out);
      CHK(hipDeviceSynchronize());
      printf("k_scatter<32> bytes %zu\n", nrec * 32);
      hipLaunchKernelGGL(k_runs<32>, dim3((unsigned)(nrec / 256)), dim3(256), 0, 0, a, nrec, out);
      CHK(hipDeviceSynchronize());
      printf("k_runs<32> bytes %zu\n", nrec * 32);
    }
    {
      const size_t nrec = ((size_t)1 << 24);     // 16 Mi records of 80 B = 1.25 GiB (power-of-two count)
      hipLaunchKernelGGL(k_scatter<80>, dim3((unsigned)(nrec / 256)), dim3(256), 0, 0, a, nrec, out);
      CHK(hipDeviceSynchronize());
      printf("k_scatter<80> bytes %zu\n", nrec * 80);
      hipLaunchKernelGGL(k_runs<80>, dim3((unsigned)(nrec / 256)), dim3(256), 0, 0, a, nrec, out);
      CHK(hipDeviceSynchronize());
      printf("k_runs<80> bytes %zu\n", nrec * 80);
    }
  }
  CHK(hipFree(a));
  CHK(hipFree(out));
  return 0;
}
