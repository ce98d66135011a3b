#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k_a(uint32_t* out, uint32_t s, int iters, unsigned long long* t) {
    uint32_t c0 = threadIdx.x ^ s, c1 = s, c2 = blockIdx.x, c3 = 7;
    long long t0 = clock64();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 10; r++) {
            uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
            uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
            uint32_t n0 = hi1 ^ c1 ^ s, n2 = hi0 ^ c3 ^ r;
            c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        }
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3;
    if (threadIdx.x == 0 && blockIdx.x == 0) *t = t1 - t0;
}
__global__ void k_b(uint32_t* out, uint32_t s, int iters, unsigned long long* t) {
    uint32_t c0 = threadIdx.x ^ s, c1 = s, c2 = blockIdx.x, c3 = 7;
    long long t0 = clock64();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 10; r++) {
            uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
            uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ s, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ r;
            c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        }
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3;
    if (threadIdx.x == 0 && blockIdx.x == 0) *t = t1 - t0;
}
int main() {
    uint32_t* o; unsigned long long* t; hipMalloc(&o, 1 << 24); hipMalloc(&t, 8);
    for (int rep = 0; rep < 2; rep++) {
    for (int v = 0; v < 2; v++) {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        int iters = 2000;
        hipEventRecord(a);
        if (v == 0) k_a<<<1024, 256>>>(o, 5, iters, t); else k_b<<<1024, 256>>>(o, 5, iters, t);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        unsigned long long tc; hipMemcpy(&tc, t, 8, hipMemcpyDeviceToHost);
        // ops: 1024 blocks*256 thr * iters * 10 rounds philox-rounds
        double rounds = 1024.0 * 256 * iters * 10;
        printf("%s: %.3f ms, %.3f Grounds/s (lanes), wave cycles per round %.2f\n", v ? "mad_u64" : "mul_lo+hi", ms, rounds / ms / 1e6, (double)tc / (iters * 10));
    }}
    return 0;
}
