// Probe of ds_read_b64_tr_b16 lane semantics: LDS holds value = 100*row + col
// (rows of 80 halves); each lane supplies the address of row (4g+q), cols 4p..
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short short4v __attribute__((ext_vector_type(4)));
__global__ void k(short* out) {
    __shared__ short tile[32 * 80];
    for (int t = threadIdx.x; t < 32 * 80; t += 64) tile[t] = (short)(100 * (t / 80) + (t % 80));
    __syncthreads();
    const int lane = threadIdx.x, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const short* a = tile + (4 * g + q) * 80 + 4 * p;
    short4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)(a));
    for (int j = 0; j < 4; ++j) out[lane * 4 + j] = v[j];
}
int main() {
    short* d; hipMalloc(&d, 64 * 4 * 2);
    k<<<1, 64>>>(d);
    short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) { printf("lane %2d:", l); for (int j = 0; j < 4; ++j) printf(" %4d", h[l*4+j]); printf("\n"); }
    return 0;
}
