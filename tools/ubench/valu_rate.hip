// Microbenchmark: issue cost of the VALU instructions the demodulator uses,
// on gfx950.  Each lane runs K independent accumulator chains (enough ILP
// to hide latency), REP iterations; cycles from s_memtime around the loop.
// Launch with W waves per SIMD (workgroup of 256*W threads on 1 CU... we use
// one workgroup per CU, 4*W waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int REP = 2048;

#define BENCH(NAME, T, INIT, OP)                                                   \
__global__ void NAME(T* out, unsigned long long* cyc, float seed) {                \
    T a0 = INIT(seed, 0), a1 = INIT(seed, 1), a2 = INIT(seed, 2), a3 = INIT(seed, 3); \
    T a4 = INIT(seed, 4), a5 = INIT(seed, 5), a6 = INIT(seed, 6), a7 = INIT(seed, 7); \
    const T b = INIT(seed, 9);                                                     \
    unsigned long long t0 = __builtin_amdgcn_s_memtime();                          \
    for (int r = 0; r < REP; ++r) {                                                \
        OP(a0, b); OP(a1, b); OP(a2, b); OP(a3, b);                                \
        OP(a4, b); OP(a5, b); OP(a6, b); OP(a7, b);                                \
    }                                                                              \
    unsigned long long t1 = __builtin_amdgcn_s_memtime();                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7; \
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                               \
}

#define IF(seed, k) ((float)(seed) + (float)(k) * 0.001f + (float)threadIdx.x * 1e-6f)
#define ID(seed, k) ((double)(seed) + (double)(k) * 0.001 + (double)threadIdx.x * 1e-9)
#define IV(seed, k) (v2f{IF(seed, k), IF(seed, k) + 0.5f})
#define OP_ADDF(a, b) a = a + b
#define OP_FMAF(a, b) a = __builtin_fmaf(a, b, b)
#define OP_ADDD(a, b) a = a + b
#define OP_FMAD(a, b) a = __builtin_fma(a, b, b)
#define OP_PKADD(a, b) a = a + b
#define OP_PKMUL(a, b) a = a * b
#define OP_CVT(a, b) a = (float)((double)a * 1.0000001)

BENCH(k_addf, float, IF, OP_ADDF)
BENCH(k_fmaf, float, IF, OP_FMAF)
BENCH(k_addd, double, ID, OP_ADDD)
BENCH(k_fmad, double, ID, OP_FMAD)
BENCH(k_pkadd, v2f, IV, OP_PKADD)
BENCH(k_pkmul, v2f, IV, OP_PKMUL)
BENCH(k_cvt, float, IF, OP_CVT)

// dependent chain: one accumulator, 8 ops per iteration
#define LAT(NAME, T, INIT, OP)                                                     \
__global__ void NAME(T* out, unsigned long long* cyc, float seed) {                \
    T a0 = INIT(seed, 0);                                                          \
    const T b = INIT(seed, 9);                                                     \
    unsigned long long t0 = __builtin_amdgcn_s_memtime();                          \
    for (int r = 0; r < REP; ++r) {                                                \
        OP(a0, b); OP(a0, b); OP(a0, b); OP(a0, b);                                \
        OP(a0, b); OP(a0, b); OP(a0, b); OP(a0, b);                                \
    }                                                                              \
    unsigned long long t1 = __builtin_amdgcn_s_memtime();                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0;                               \
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                               \
}
LAT(l_addf, float, IF, OP_ADDF)
LAT(l_fmaf, float, IF, OP_FMAF)
LAT(l_pkadd, v2f, IV, OP_PKADD)
LAT(l_addd, double, ID, OP_ADDD)
LAT(l_fmad, double, ID, OP_FMAD)

template <typename K, typename T>
void run(const char* name, K kern, int waves_per_simd, int ops_per_iter) {
    int threads = 256 * waves_per_simd > 1024 ? 1024 : 256 * waves_per_simd;
    int blocks_per_cu = (256 * waves_per_simd) / threads;
    int cus = 256;
    int blocks = cus * blocks_per_cu;
    T* out; unsigned long long* cyc;
    hipMalloc(&out, sizeof(T) * blocks * threads);
    hipMalloc(&cyc, sizeof(unsigned long long) * blocks);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0f);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0f);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(blocks);
    hipMemcpy(c.data(), cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    double avg = 0; for (auto v : c) avg += v; avg /= blocks;
    // wave-instructions issued per SIMD in the loop
    double instr_per_simd = (double)REP * 8 * ops_per_iter * waves_per_simd;
    printf("%-8s waves/SIMD=%d  cycles/loop=%.0f  cycles per wave-instr per SIMD=%.2f  (wall %.3f ms)\n",
           name, waves_per_simd, avg, avg / instr_per_simd, ms);
    hipFree(out); hipFree(cyc);
}

int main() {
    for (int w : {1, 2, 4}) {
        run<decltype(&k_addf), float>("add_f32", k_addf, w, 1);
        run<decltype(&k_fmaf), float>("fma_f32", k_fmaf, w, 1);
        run<decltype(&k_pkadd), v2f>("pk_add", k_pkadd, w, 1);
        run<decltype(&k_pkmul), v2f>("pk_mul", k_pkmul, w, 1);
        run<decltype(&k_addd), double>("add_f64", k_addd, w, 1);
        run<decltype(&k_fmad), double>("fma_f64", k_fmad, w, 1);
        run<decltype(&k_cvt), float>("cvt+mul", k_cvt, w, 3);
    }
    for (int w : {1, 2}) {
        run<decltype(&l_addf), float>("LAT add_f32", l_addf, w, 1);
        run<decltype(&l_fmaf), float>("LAT fma_f32", l_fmaf, w, 1);
        run<decltype(&l_pkadd), v2f>("LAT pk_add", l_pkadd, w, 1);
        run<decltype(&l_addd), double>("LAT add_f64", l_addd, w, 1);
        run<decltype(&l_fmad), double>("LAT fma_f64", l_fmad, w, 1);
    }
    return 0;
}
