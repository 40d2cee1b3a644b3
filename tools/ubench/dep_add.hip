// Latency of a dependent f32 add chain on one lane (the modulator's phase
// walk, k_mod_accumulate, is 8,448 of them at SF 7): registers only, vs the
// same chain fed from global memory in 64-sample blocks (the shipped
// kernel's loads), each timed after an idle gap as the per-packet loop sees
// it.  Timing aid only.  hipcc --offload-arch=gfx950 -O3 dep_add.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>

__global__ void k_chain_regs(float* out, int n, float step) {
    float ph = 0.0f, f = step;
    for (int i = 0; i < n; ++i) {
        ph += f;
        f += 1.0e-7f;  // independent of ph (the f sequence is precomputed in the walk)
    }
    out[0] = ph;
}

__global__ void k_chain_mem(float* io, int n) {
    float ph = 0.0f;
    for (int i = 0; i < n; i += 4) {
        const float4 b = *reinterpret_cast<const float4*>(io + i);
        float4 o;
        ph += b.x; o.x = ph;
        ph += b.y; o.y = ph;
        ph += b.z; o.z = ph;
        ph += b.w; o.w = ph;
        *reinterpret_cast<float4*>(io + i) = o;
    }
}

int main() {
    const int n = 8448;
    float* d;
    hipMalloc(&d, n * sizeof(float) * 2);
    hipMemset(d, 0, n * sizeof(float) * 2);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 6; ++rep) {
        std::this_thread::sleep_for(std::chrono::milliseconds(rep < 3 ? 20 : 0));
        float ms1 = 0, ms2 = 0;
        hipEventRecord(a);
        hipLaunchKernelGGL(k_chain_regs, dim3(1), dim3(64), 0, 0, d, n, 0.01f);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms1, a, b);
        std::this_thread::sleep_for(std::chrono::milliseconds(rep < 3 ? 20 : 0));
        hipEventRecord(a);
        hipLaunchKernelGGL(k_chain_mem, dim3(1), dim3(64), 0, 0, d, n);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms2, a, b);
        printf("%s: registers %.1f us (%.2f ns/add), loads+stores %.1f us (%.2f ns/add)\n",
               rep < 3 ? "after 20 ms idle" : "back to back", ms1 * 1e3, ms1 * 1e6 / n, ms2 * 1e3, ms2 * 1e6 / n);
    }
    return 0;
}
