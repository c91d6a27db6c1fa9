// store_bw.hip -- the HBM write roofline the rollout kernel's row stores are priced against.
// A store-only stream over a buffer larger than the MALL, in the rollout's access shapes:
//   lines : each wave instruction writes 1 KiB contiguous (64 lanes x 16 B), waves stride
//           through the buffer (the best case: whole 128-B lines per instruction)
//   rows16: each instruction writes 16 rows x 64 B (lane (r, q): row r, bytes 16 q .. of the
//           row's 64-B piece) -- the agent-tile obs stores (rows 1 KiB apart), the piece
//           advancing with the next instruction
//   nt    : `lines` with nontemporal stores
// Build:  hipcc -O3 --offload-arch=gfx950 tools/store_bw.hip -o build/store_bw
// Run:    build/store_bw [GiB=4]   -> one line per shape: GB/s (best of 5, HIP events)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) st_lines(f32x4 *p, size_t n4, int iters) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const f32x4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) p[i] = v;
    (void)iters;
}

__global__ void __launch_bounds__(256) st_lines_nt(f32x4 *p, size_t n4, int iters) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const f32x4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
        __builtin_nontemporal_store(v, p + i);
    (void)iters;
}

// one wave owns 16 rows of 1 KiB (16 KiB tiles); instruction k writes bytes 64 k .. 64 k + 63
// of each of its 16 rows: lane (r, q) -> row r, 16 B at 64 k + 16 q
__global__ void __launch_bounds__(256) st_rows16(f32x4 *p, size_t n4, int iters) {
    const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    const size_t tiles = n4 / (16 * 64);  // 16 rows x 64 f32x4 per tile
    const f32x4 v = {1.f, 2.f, 3.f, (float)lane};
    for (size_t t = wave; t < tiles; t += nwaves) {
        f32x4 *row = p + t * 16 * 64 + (size_t)r * 64;
#pragma unroll 4
        for (int k = 0; k < 16; ++k) row[4 * k + q] = v;
    }
    (void)iters;
}

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 4.0;
    const size_t bytes = (size_t)(gib * (1ull << 30)) / (16 * 64 * 16) * (16 * 64 * 16);
    const size_t n4 = bytes / 16;
    f32x4 *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Shape {
        const char *name;
        void (*k)(f32x4 *, size_t, int);
    } shapes[] = {{"lines", st_lines}, {"rows16", st_rows16}, {"nt", st_lines_nt}};
    for (int occ : {4, 8, 16}) {
        const unsigned grid = (unsigned)(cus * occ);
        for (const Shape &sh : shapes) {
            float best = 1e30f;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(e0, 0);
                hipLaunchKernelGGL(sh.k, dim3(grid), dim3(256), 0, 0, p, n4, 1);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms = 0.f;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep > 0 && ms < best) best = ms;  // rep 0 warms up
            }
            printf("{\"shape\": \"%s\", \"workgroups_per_cu\": %d, \"bytes\": %zu, \"ms\": %.4f, \"GBps\": %.1f}\n",
                   sh.name, occ, bytes, best, bytes / (best * 1e-3) / 1e9);
        }
    }
    hipFree(p);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
