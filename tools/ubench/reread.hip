// Microbenchmark: is a second read of each frame, one frame later per wave
// (the fused kernel's max-abs scan + symbol pass), served on-die (Infinity
// Cache) or does it cost HBM bandwidth?  Timing aid only.
//   reread <frames> <frame_kb> <mode>   mode 0: each frame once
//                                        mode 1: each frame twice (scan k+1, then re-read k)
//                                        mode 2: mode 1 with the re-read two frames later
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256, 2) void k_stream(const float4* __restrict__ iq, unsigned frames,
                                                unsigned f4_per_frame, unsigned waves, int mode,
                                                float* out) {
    const unsigned lane = threadIdx.x & 63, w = blockIdx.x * 4 + (threadIdx.x >> 6);
    float acc = 0.0f;
    auto pass = [&](unsigned f) {
        const float4* p = iq + (size_t)f * f4_per_frame;
        unsigned b = 0;
        for (; b + 64 * 16 <= f4_per_frame; b += 64 * 16) {  // unconditional rounds
            float4 v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = p[b + u * 64 + lane];
#pragma unroll
            for (int u = 0; u < 16; ++u) acc = fmaxf(acc, fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w)));
        }
        for (unsigned j = b + lane; j < f4_per_frame; j += 64) {
            const float4 v = p[j];
            acc = fmaxf(acc, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
        }
    };
    const int lag = mode == 2 ? 2 : 1;
    for (unsigned f = w, k = 0; f < frames + (mode ? lag * waves : 0); f += waves, ++k) {
        if (f < frames) pass(f);
        if (mode && k >= (unsigned)lag) pass(f - lag * waves);
    }
    if (acc == 12345.0f) out[w] = acc;
}

int main(int argc, char** argv) {
    const unsigned frames = argc > 1 ? atoi(argv[1]) : 65536;
    const unsigned kb = argc > 2 ? atoi(argv[2]) : 66;
    const int mode = argc > 3 ? atoi(argv[3]) : 0;
    const unsigned f4 = kb * 1024 / 16;
    float4* d;
    float* o;
    hipMalloc(&d, (size_t)frames * f4 * 16);
    hipMalloc(&o, 1 << 20);
    hipMemset(d, 0, (size_t)frames * f4 * 16);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int per = argc > 4 ? atoi(argv[4]) : 2;
    const unsigned blocks = cus * per, waves = blocks * 4;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(256), 0, 0, d, frames, f4, waves, mode, o);
    hipEventRecord(a);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(256), 0, 0, d, frames, f4, waves, mode, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double bytes = (double)frames * f4 * 16;
    printf("mode %d frames %u x %u KB: %.3f ms  unique %.2f TB/s  delivered %.2f TB/s\n", mode, frames, kb, ms,
           bytes / ms / 1e9, bytes * (mode ? 2 : 1) / ms / 1e9);
    return 0;
}
