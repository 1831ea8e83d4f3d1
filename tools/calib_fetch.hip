// tools/calib_fetch.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the
// access widths of this engine's gather/scatter kernels (MI355X_MICROARCH.md §HBM: only the
// 16-B/lane streaming read (x2) and the streaming store (x1) are calibrated there).
//
// Every kernel touches a known set of DISTINCT lines of a 1 GiB buffer (past the 256 MiB
// Infinity Cache, lines touched once), so the HBM-side bytes are known exactly:
//   stream16   : 16 B per lane, sequential, 1 GiB read
//   gather2    : one 2-B read in each of 2^23 distinct 128-B lines (a bijective line order)
//   gather8    : one 8-B read per line, same lines
//   gather2x4  : four 2-B reads in each line (adjacent lanes, same line)
//   scatter2   : one 2-B store in each of 2^23 distinct 128-B lines
//   scatter16  : one 16-B store in each line
// tools/calib_fetch.sh runs it under one --pmc pass per counter and prints counter / known.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr size_t kBytes = size_t(1) << 30;
constexpr uint32_t kLines = uint32_t(kBytes / 128);        // 2^23 lines of 128 B

__device__ inline uint32_t line_of(uint32_t i) { return (i * 2654435761u) & (kLines - 1); }

__global__ void stream16(const uint4* __restrict__ in, uint32_t* out) {
    const size_t n = kBytes / 16;
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <class T>
__global__ void gather(const T* __restrict__ in, uint32_t per_line, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kLines * per_line) return;
    const uint32_t line = line_of(i / per_line), k = i % per_line;
    const T v = in[(size_t)line * (128 / sizeof(T)) + k];
    if (v == (T)0x1234) out[0] = 1;              // (never: the buffer holds 0x01 bytes)
}

template <class T>
__global__ void scatter(T* __restrict__ buf) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kLines) return;
    buf[(size_t)line_of(i) * (128 / sizeof(T))] = T{};
}

int main() {
    char* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, kBytes);
    (void)hipDeviceSynchronize();
    const dim3 b(256);
    hipLaunchKernelGGL(stream16, dim3(4096), b, 0, 0, (const uint4*)buf, out);
    hipLaunchKernelGGL(gather<uint16_t>, dim3(kLines / 256), b, 0, 0, (const uint16_t*)buf, 1u, out);
    hipLaunchKernelGGL(gather<uint64_t>, dim3(kLines / 256), b, 0, 0, (const uint64_t*)buf, 1u, out);
    hipLaunchKernelGGL(gather<uint16_t>, dim3(kLines / 64), b, 0, 0, (const uint16_t*)buf, 4u, out);
    hipLaunchKernelGGL(scatter<uint16_t>, dim3(kLines / 256), b, 0, 0, (uint16_t*)buf);
    hipLaunchKernelGGL(scatter<uint4>, dim3(kLines / 256), b, 0, 0, (uint4*)buf);
    (void)hipDeviceSynchronize();
    std::printf("lines %u, bytes %zu\n", kLines, kBytes);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
