// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the load
// and store widths the decode kernels use (MI355X_MICROARCH.md: FETCH_SIZE is
// calibrated only for 16 B/lane streaming reads; "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Each kernel touches a known number of bytes of a 1 GiB buffer (4x the
// 256 MiB Infinity Cache, so nothing is served on-die across launches):
//   rd16   uint4 per lane, coalesced                 (k_decode_staged staging)
//   rd4    one dword per lane, coalesced             (k_inflate input ring refill)
//   rd1    one byte per lane, coalesced
//   rd4s64 one dword per 64 B, each line once        (k_inflate far-history reads)
//   rd4s128 one dword per 128 B
//   wr16 / wr4 / wr1  stores of the same widths
// Usage: calib_fetch   (prints kernel name -> algorithmic bytes touched)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void rd16(const uint4* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t a = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = p[i];
        a ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (a == 0x12345678u) out[0] = a;
}
__global__ void rd4(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t a = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a ^= p[i];
    if (a == 0x12345678u) out[0] = a;
}
__global__ void rd1(const uint8_t* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t a = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a += p[i];
    if (a == 0x12345678u) out[0] = a;
}
template <int STRIDE>
__global__ void rd4s(const uint8_t* __restrict__ p, size_t lines, uint32_t* out) {
    uint32_t a = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x) {
        // scatter the lines over the buffer (odd multiplier: a permutation of 0..lines-1 for power-of-2 lines)
        size_t l = (i * 2654435761ull) & (lines - 1);
        a ^= *reinterpret_cast<const uint32_t*>(p + l * STRIDE);
    }
    if (a == 0x12345678u) out[0] = a;
}
__global__ void wr16(uint4* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__global__ void wr4(uint32_t* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)i;
}
__global__ void wr1(uint8_t* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint8_t)i;
}

int main() {
    const size_t B = size_t(1) << 30;
    uint8_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, B));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 1, B));
    const int grid = 256 * 8 * 4, blk = 256;
    for (int rep = 0; rep < 3; ++rep) {
        rd16<<<grid, blk>>>((const uint4*)buf, B / 16, out);
        rd4<<<grid, blk>>>((const uint32_t*)buf, B / 4, out);
        rd1<<<grid, blk>>>(buf, B, out);
        rd4s<64><<<grid, blk>>>(buf, B / 64, out);
        rd4s<128><<<grid, blk>>>(buf, B / 128, out);
        wr16<<<grid, blk>>>((uint4*)buf, B / 16);
        wr4<<<grid, blk>>>((uint32_t*)buf, B / 4);
        wr1<<<grid, blk>>>(buf, B);
        CK(hipDeviceSynchronize());
    }
    std::printf("{\"rd16\": %zu, \"rd4\": %zu, \"rd1\": %zu, \"rd4s64_lines\": %zu, \"rd4s128_lines\": %zu, "
                "\"wr16\": %zu, \"wr4\": %zu, \"wr1\": %zu}\n",
                B, B, B, B / 64, B / 128, B, B, B);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
