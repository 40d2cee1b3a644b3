// Microbenchmark: does a second wave per SIMD raise packed-f32 VALU
// throughput?  256 workgroups (one per CU) of 256 threads (1 wave / SIMD)
// or 512 threads (2 waves / SIMD), each wave runs the same fixed work:
// REP iterations of ILP independent v_pk_fma_f32 chains.  Wall time by HIP
// events over a long loop (launch overhead negligible).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));
template <int ILP>
__global__ void k(v2f* out, int rep, float seed) {
    v2f a[ILP];
    for (int i = 0; i < ILP; ++i) a[i] = v2f{seed + i, seed - i} + (float)threadIdx.x * 1e-6f;
    const v2f b = {0.999f, 1.001f}, c = {1e-7f, -1e-7f};
    for (int r = 0; r < rep; ++r) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int i = 0; i < ILP; ++i) a[i] = __builtin_elementwise_fma(a[i], b, c);
    }
    v2f s = a[0];
    for (int i = 1; i < ILP; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int ILP>
void run(int threads, int rep) {
    v2f* o;
    hipMalloc(&o, sizeof(v2f) * 256 * 1024);
    hipLaunchKernelGGL(k<ILP>, dim3(256), dim3(threads), 0, 0, o, rep, 1.0f);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<ILP>, dim3(256), dim3(threads), 0, 0, o, rep, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double instr_per_simd = (double)rep * 8 * ILP * (threads / 256);
    printf("ILP %d threads %d (waves/SIMD %d): %.3f ms, %.2f ns per wave-instr per SIMD, %.2f cycles at 2.4 GHz\n", ILP,
           threads, threads / 256, ms, ms * 1e6 / instr_per_simd, ms * 1e6 / instr_per_simd * 2.4);
    hipFree(o);
}
int main() {
    const int rep = 20000;
    for (int t : {256, 512, 768, 1024}) run<8>(t, rep);
    for (int t : {256, 512}) run<2>(t, rep);
    for (int t : {256, 512}) run<1>(t, rep);
    printf("SIMD2_DONE\n");
    return 0;
}
