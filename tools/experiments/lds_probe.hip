// LDS latency by address region (gfx950): one workgroup of one wave per launch walks a dependent
// chain of ds_read_b32 inside a 16 KB window at each offset; cycles per read from s_memtime.
// build: hipcc --offload-arch=gfx950 -O3 tools/lds_probe.hip -o tools/lds_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_walk(unsigned* out, unsigned window_base_words, unsigned steps) {
    extern __shared__ unsigned lds[];
    const unsigned lane = threadIdx.x;
    // fill the whole 160 KB with a permutation-ish pointer chain inside each 16 KB window
    for (unsigned i = lane; i < 40960; i += 64) {
        const unsigned win = i & ~4095u;
        lds[i] = win + ((i * 2654435761u + 12345u) & 4095u);
    }
    __syncthreads();
    unsigned p = window_base_words + ((lane * 67u) & 4095u);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (unsigned s = 0; s < steps; ++s) p = lds[p];
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[0] = (unsigned)(t1 - t0);
    out[1 + lane] = p;
}

int main() {
    unsigned* d;
    hipMalloc(&d, 4096);
    hipFuncSetAttribute((const void*)k_walk, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const unsigned offs_kb[] = {0, 32, 64, 96, 112, 128, 136, 144};
    for (unsigned o : offs_kb) {
        const unsigned steps = 4096;
        unsigned best = ~0u;
        for (int rep = 0; rep < 5; ++rep) {
            k_walk<<<1, 64, 160 * 1024>>>(d, o * 256, steps);
            unsigned h = 0;
            hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
            best = h < best ? h : best;
        }
        printf("window at %3u KB: %.1f cycles per dependent ds_read_b32\n", o, (double)best / steps);
    }
    hipFree(d);
    return 0;
}
