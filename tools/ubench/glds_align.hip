// Microtest: global_load_lds_dwordx4 (LDS-DMA, 16 B per lane) from source
// addresses that are only 8-byte aligned (odd complex-sample offsets), as the
// SF 11-12 wave kernel issues for odd time shifts / odd frame lengths; and
// the instruction's immediate offset, which must move the global source and
// the LDS destination alike (k_glds_imm: one base, offsets 0..3 KiB).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void g_void;

__global__ void k_glds(const float2* src, float2* dst, int off) {
    __shared__ float2 buf[1024];
    const int lane = threadIdx.x;
    for (int r = 0; r < 8; ++r) {
        const float2* g = src + off + 128 * r + 2 * lane;
        __builtin_amdgcn_global_load_lds((g_void*)g, (lds_void*)(buf + 128 * r), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    for (int i = lane; i < 1024; i += 64) dst[i] = buf[i];
}

__global__ void k_glds_imm(const float2* src, float2* dst, int off) {
    __shared__ float2 buf[1024];
    const int lane = threadIdx.x;
    for (int r = 0; r < 8; r += 4) {
        const float2* g = src + off + 128 * r + 2 * lane;
        __builtin_amdgcn_global_load_lds((g_void*)g, (lds_void*)(buf + 128 * r), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((g_void*)g, (lds_void*)(buf + 128 * r), 16, 1024, 0);
        __builtin_amdgcn_global_load_lds((g_void*)g, (lds_void*)(buf + 128 * r), 16, 2048, 0);
        __builtin_amdgcn_global_load_lds((g_void*)g, (lds_void*)(buf + 128 * r), 16, 3072, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    for (int i = lane; i < 1024; i += 64) dst[i] = buf[i];
}

int main() {
    const int n = 4096;
    std::vector<float2> h(n);
    for (int i = 0; i < n; ++i) h[i] = make_float2((float)i, -(float)i);
    float2 *d, *o;
    hipMalloc(&d, n * sizeof(float2));
    hipMalloc(&o, 1024 * sizeof(float2));
    hipMemcpy(d, h.data(), n * sizeof(float2), hipMemcpyHostToDevice);
    int bad = 0;
    for (int imm = 0; imm < 2; ++imm)
    for (int off : {0, 1, 2, 3, 7}) {
        hipMemset(o, 0, 1024 * sizeof(float2));
        if (imm) hipLaunchKernelGGL(k_glds_imm, dim3(1), dim3(64), 0, 0, d, o, off);
        else hipLaunchKernelGGL(k_glds, dim3(1), dim3(64), 0, 0, d, o, off);
        std::vector<float2> r(1024);
        hipMemcpy(r.data(), o, 1024 * sizeof(float2), hipMemcpyDeviceToHost);
        int e = 0;
        for (int i = 0; i < 1024; ++i) e += r[i].x != (float)(i + off) || r[i].y != -(float)(i + off);
        printf("%s offset %d samples: %d mismatches\n", imm ? "imm" : "base", off, e);
        bad += e;
    }
    printf(bad ? "GLDS_ALIGN_FAIL\n" : "GLDS_ALIGN_OK\n");
    return bad != 0;
}
