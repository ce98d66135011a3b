// FETCH_SIZE / WRITE_SIZE calibration for the access shapes of the node-round
// kernels (MI355X_MICROARCH.md: "other access widths are uncalibrated").
// Each kernel touches a known number of distinct 64-B lines of a 4 GiB
// buffer (far past the 256 MiB Infinity Cache), so the counters can be
// divided by the known byte count:
//   k_stream   16 B per lane, coalesced              (the guide's calibrated case)
//   k_rand4    one random dword per lane              (flag / partition bytes, ids)
//   k_rand64   one random 64-B record per 16 lanes    (message records, rows)
//   k_wrand64  one random 64-B record store per 16 lanes
// Build: hipcc -O3 --offload-arch=gfx950 calib_fetch.hip -o calib_fetch
// Run:   rocprofv3 --pmc FETCH_SIZE -- ./calib_fetch   (WRITE_SIZE in its own pass)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t BUF = 4ull << 30;                 // bytes
constexpr uint32_t LINES = (uint32_t)(BUF / 64);   // 64-B lines
constexpr uint32_t N = 1u << 24;                   // accesses per kernel

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void k_stream(const uint4* __restrict__ in, uint32_t n16, uint32_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint4 v = i < n16 ? in[i] : make_uint4(0, 0, 0, 0);
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = i;
}
__global__ void k_rand4(const uint32_t* __restrict__ in, uint32_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    uint32_t line = mix(i) % LINES;               // distinct lines with high probability
    uint32_t v = in[(size_t)line * 16 + (i & 15)];
    if (v == 0x12345678u) out[0] = i;
}
__global__ void k_rand64(const uint32_t* __restrict__ in, uint32_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t rec = i >> 4;
    if (rec >= N / 16) return;
    uint32_t line = mix(rec + 0x9e3779b9u) % LINES;
    uint32_t v = in[(size_t)line * 16 + (i & 15)];
    if (v == 0x12345678u) out[0] = i;
}
__global__ void k_wrand64(uint32_t* __restrict__ buf) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t rec = i >> 4;
    if (rec >= N / 16) return;
    uint32_t line = mix(rec + 0x7f4a7c15u) % LINES;
    buf[(size_t)line * 16 + (i & 15)] = i;
}

int main() {
    uint32_t *buf = nullptr, *out = nullptr;
    if (hipMalloc(&buf, BUF) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 1, BUF);
    hipDeviceSynchronize();
    const uint32_t n16 = N;                        // 16-B pieces streamed: N * 16 B
    for (int rep = 0; rep < 3; rep++) {
        k_stream<<<n16 / 256, 256>>>(reinterpret_cast<const uint4*>(buf), n16, out);
        k_rand4<<<N / 256, 256>>>(buf, out);
        k_rand64<<<N / 256, 256>>>(buf, out);
        k_wrand64<<<N / 256, 256>>>(buf);
    }
    hipDeviceSynchronize();
    std::printf("known bytes per dispatch: k_stream %u, k_rand4 %u lines (x64 B = %u), "
                "k_rand64 %u records (x64 B = %u), k_wrand64 %u records (x64 B = %u)\n",
                n16 * 16, N, N * 64, N / 16, N / 16 * 64, N / 16, N / 16 * 64);
    hipFree(buf); hipFree(out);
    return 0;
}
