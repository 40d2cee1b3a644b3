// Experiment (timing and layout check only, not the library): a 128-point
// DFT of 8 symbols per wavefront on the matrix cores, 128 = 16 x 8.
//   stage 1: P[k1][n2] = sum_n1 x[8 n1 + n2] W16^(n1 k1)     (MFMA, x as A)
//   twiddle: P[k1][n2] *= W128^(n2 k1)                         (VALU, f32)
//   stage 2: X[k1 + 16 k2] = sum_n2 P[k1][n2] W8^(n2 k2)      (MFMA, P as B)
// v_mfma_f32_16x16x32_f16, complex arithmetic real-ified (K = 32 = 16
// complex).  Stage 1's accumulator is stage 2's B operand in place: its
// column (k1) is on the lane and its rows (s, n2) in the registers, so the
// product over n2 needs no lane movement.  Two symbols per MFMA tile (rows
// s, n2), stage 2's A block-diagonal over s.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o mfma_dft.so mfma_dft.hip
#include <hip/hip_runtime.h>

#include <cmath>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

namespace {

constexpr float kPi = 3.14159265358979f;

struct Consts {  // per lane, built once
    h8 b1r, b1i, a2r, a2i;
    float tr[4], ti[4];
};

__device__ Consts make_consts(int l) {
    Consts K;
    const int col = l & 15, q = l >> 4, row = l & 15;
    for (int j = 0; j < 8; ++j) {
        const int c = j & 1;
        // stage 1 B: k = 8q + j <-> (n1 = 4q + j/2, c), column k1 = col
        {
            const int n1 = 4 * q + (j >> 1);
            const double a = -2.0 * M_PI * (double)(n1 * col) / 16.0;
            const float wr = (float)cos(a), wi = (float)sin(a);
            K.b1r[j] = (_Float16)(c == 0 ? wr : -wi);
            K.b1i[j] = (_Float16)(c == 0 ? wi : wr);
        }
        // stage 2 A: row (s', k2) = row, k = 8q + j <-> (r = 4q + j/2 -> s = r>>3, n2 = r&7; c)
        {
            const int sp = row >> 3, k2 = row & 7, r = 4 * q + (j >> 1), s = r >> 3, n2 = r & 7;
            const double a = -2.0 * M_PI * (double)(n2 * k2) / 8.0;
            const float vr = (float)cos(a), vi = (float)sin(a);
            const float on = s == sp ? 1.0f : 0.0f;
            K.a2r[j] = (_Float16)(on * (c == 0 ? vr : -vi));
            K.a2i[j] = (_Float16)(on * (c == 0 ? vi : vr));
        }
    }
    for (int i = 0; i < 4; ++i) {
        const int n2 = 4 * (q & 1) + i;
        const double a = -2.0 * M_PI * (double)(n2 * col) / 128.0;
        K.tr[i] = (float)cos(a);
        K.ti[i] = (float)sin(a);
    }
    return K;
}

// one tile: symbols s0, s0 + 1 from `x` (natural order, 128 complex each)
__device__ __forceinline__ void dft_tile(const float2* __restrict__ x, int s0, const Consts& K, int l,
                                         f4& xr, f4& xi) {
    const int row = l & 15, q = l >> 4;
    const int s = s0 + (row >> 3), n2 = row & 7;
    h8 a;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
        const float2 v = x[s * 128 + 8 * (4 * q + jj) + n2];
        a[2 * jj] = (_Float16)v.x;
        a[2 * jj + 1] = (_Float16)v.y;
    }
    const f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
    const f4 cr = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, K.b1r, z, 0, 0, 0);
    const f4 ci = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, K.b1i, z, 0, 0, 0);
    h8 b;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float pr = cr[i] * K.tr[i] - ci[i] * K.ti[i];
        const float pi = cr[i] * K.ti[i] + ci[i] * K.tr[i];
        b[2 * i] = (_Float16)pr;
        b[2 * i + 1] = (_Float16)pi;
    }
    xr = __builtin_amdgcn_mfma_f32_16x16x32_f16(K.a2r, b, z, 0, 0, 0);
    xi = __builtin_amdgcn_mfma_f32_16x16x32_f16(K.a2i, b, z, 0, 0, 0);
}

__global__ __launch_bounds__(64) void k_mfma_dft128(const float2* __restrict__ x, float2* __restrict__ out,
                                                    int groups) {
    const int l = threadIdx.x;
    const Consts K = make_consts(l);
    const int q = l >> 4, col = l & 15;
    for (int g = blockIdx.x; g < groups; g += gridDim.x) {
        const float2* xs = x + (size_t)g * 8 * 128;
        float2* os = out + (size_t)g * 8 * 128;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            f4 xr, xi;
            dft_tile(xs, 2 * t, K, l, xr, xi);
            const int s = 2 * t + (q >> 1);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int k2 = 4 * (q & 1) + i;
                os[s * 128 + col + 16 * k2] = float2{xr[i], xi[i]};
            }
        }
    }
}

}  // namespace

extern "C" int mfma_dft128(const float* x, float* out, int symbols, void* stream) {
    if (symbols % 8) return -22;
    const int groups = symbols / 8;
    const int grid = groups < 4096 ? groups : 4096;
    hipLaunchKernelGGL(k_mfma_dft128, dim3(grid), dim3(64), 0, (hipStream_t)stream,
                       reinterpret_cast<const float2*>(x), reinterpret_cast<float2*>(out), groups);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
