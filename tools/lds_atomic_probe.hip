// LDS atomic throughput probe (gfx950): cycles per wave-instruction of
// ds_add_f32 / ds_add_u32 / ds_add_u64 / ds_pk_add_f16 / ds_write_b32 on random and
// conflict-free addresses. Build: hipcc --offload-arch=gfx950 -O3 -o build/lds_probe tools/lds_atomic_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
constexpr int N = 1024;  // operations per thread

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <int MODE, bool RANDOM>
__global__ void __launch_bounds__(512) k(float* out) {
    __shared__ float acc[16384];
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) acc[i] = 0.f;
    __syncthreads();
    uint32_t s = mix(threadIdx.x * 7919u + blockIdx.x * 104729u);
    for (int i = 0; i < N; ++i) {
        const uint32_t a = RANDOM ? (mix(s + i) & 16383u) : ((threadIdx.x + i * 64u) & 16383u);
        if (MODE == 0) atomicAdd(&acc[a], 1.0f);
        if (MODE == 1) atomicAdd(reinterpret_cast<uint32_t*>(acc) + a, 1u);
        if (MODE == 2) __builtin_amdgcn_ds_atomic_fadd_v2f16(
            (__attribute__((address_space(3))) h2*)(reinterpret_cast<h2*>(acc) + a), h2{1.0f, 1.0f});
        if (MODE == 3) acc[a] = (float)i;
        if (MODE == 4) atomicAdd(reinterpret_cast<unsigned long long*>(acc) + (a & 8191u), 1ull);
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = acc[blockIdx.x & 16383];
}

template <int MODE, bool RANDOM>
void run(const char* name, float* out) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int blocks = 256 * 2;
    k<MODE, RANDOM><<<blocks, 512>>>(out);
    hipEventRecord(a);
    k<MODE, RANDOM><<<blocks, 512>>>(out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double wave_instr_per_cu = (double)blocks * 512 / 64 * N / 256;
    printf("%-28s %8.1f us  %6.1f cycles/wave-instr/CU (2.4GHz)\n", name, ms * 1e3, ms * 1e-3 * 2.4e9 / wave_instr_per_cu);
}

int main() {
    float* out; hipMalloc(&out, 4096 * 4);
    run<0, true>("ds_add_f32 random", out);
    run<0, false>("ds_add_f32 distinct", out);
    run<1, true>("ds_add_u32 random", out);
    run<1, false>("ds_add_u32 distinct", out);
    run<2, true>("ds_pk_add_f16 random", out);
    run<2, false>("ds_pk_add_f16 distinct", out);
    run<4, true>("ds_add_u64 random", out);
    run<4, false>("ds_add_u64 distinct", out);
    run<3, true>("ds_write_b32 random", out);
    run<3, false>("ds_write_b32 distinct", out);
    return 0;
}
