// store_bw.hip -- the HBM write ceiling the rollout kernel's row stores are priced against
// (bench.py store_ceiling).  Store-only streams, one launch each, in the rollout's access shapes:
//   lines  : each wave instruction writes 1 KiB contiguous (64 lanes x 16 B), waves grid-stride
//            through the buffer (whole 128-B lines per instruction)
//   rows16 : each instruction writes 16 rows x 64 B (lane (r, q): row r, bytes 16 q .. of the
//            row's 64-B piece) -- the agent-tile obs stores (rows 1 KiB apart), the piece
//            advancing with the next instruction
//   nt     : `lines` with nontemporal stores
//   reuse  : `lines` over a 256 MiB buffer rewritten `passes` times in the launch -- the REDA Q
//            buffer's pattern (asg_step_forward rewrites the same 256 MiB every step): the
//            256 MiB Infinity Cache (MALL) absorbs much of it, so it is NOT an HBM rate
// The HBM shapes write a buffer far larger than the MALL (default 32 GiB, ~the bytes one
// whole-episode rollout launch writes in 7 ms), so launch ramp-up and tail are < 2 % of the
// time; workgroups of 256 threads, 2 .. 8 per CU (8 = 32 waves per CU, the limit).
// Build:  hipcc -O3 --offload-arch=gfx950 tools/store_bw.hip -o build/store_bw
// Run:    build/store_bw [GiB=32]  -> one JSON line per (shape, workgroups per CU): GB/s (best of 4)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) st_lines(f32x4 *p, size_t n4, int passes) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const f32x4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
    for (int it = 0; it < passes; ++it)
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) p[i] = v;
}

__global__ void __launch_bounds__(256) st_lines_nt(f32x4 *p, size_t n4, int passes) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const f32x4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
    for (int it = 0; it < passes; ++it)
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
            __builtin_nontemporal_store(v, p + i);
}

// one wave owns 16 rows of 1 KiB (16 KiB tiles); instruction k writes bytes 64 k .. 64 k + 63
// of each of its 16 rows: lane (r, q) -> row r, 16 B at 64 k + 16 q
__global__ void __launch_bounds__(256) st_rows16(f32x4 *p, size_t n4, int passes) {
    const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    const size_t tiles = n4 / (16 * 64);  // 16 rows x 64 f32x4 per tile
    const f32x4 v = {1.f, 2.f, 3.f, (float)lane};
    for (int it = 0; it < passes; ++it)
        for (size_t t = wave; t < tiles; t += nwaves) {
            f32x4 *row = p + t * 16 * 64 + (size_t)r * 64;
#pragma unroll 4
            for (int k = 0; k < 16; ++k) row[4 * k + q] = v;
        }
}

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 32.0;
    const size_t tile = 16 * 64 * 16;
    const size_t bytes = (size_t)(gib * (1ull << 30)) / tile * tile;
    const size_t reuse_bytes = 256ull << 20;
    f32x4 *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        fprintf(stderr, "hipMalloc of %zu bytes failed\n", bytes);
        return 1;
    }
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct Shape {
        const char *name;
        void (*k)(f32x4 *, size_t, int);
        size_t bytes;
        int passes;
    } shapes[] = {{"lines", st_lines, bytes, 1},
                  {"rows16", st_rows16, bytes, 1},
                  {"nt", st_lines_nt, bytes, 1},
                  {"reuse", st_lines, reuse_bytes, (int)(bytes / reuse_bytes)}};
    for (int occ : {2, 4, 8}) {
        const unsigned grid = (unsigned)(cus * occ);
        for (const Shape &sh : shapes) {
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                (void)hipEventRecord(e0, 0);
                hipLaunchKernelGGL(sh.k, dim3(grid), dim3(256), 0, 0, p, sh.bytes / 16, sh.passes);
                (void)hipEventRecord(e1, 0);
                (void)hipEventSynchronize(e1);
                float ms = 0.f;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (rep > 0 && ms < best) best = ms;  // rep 0 warms up
            }
            const double moved = (double)sh.bytes * sh.passes;
            printf("{\"shape\": \"%s\", \"workgroups_per_cu\": %d, \"bytes\": %.0f, \"buffer_bytes\": %zu, "
                   "\"ms\": %.4f, \"GBps\": %.1f, \"hbm\": %s}\n",
                   sh.name, occ, moved, sh.bytes, best, moved / (best * 1e-3) / 1e9,
                   sh.bytes > reuse_bytes ? "true" : "false");
            fflush(stdout);
        }
    }
    (void)hipFree(p);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
