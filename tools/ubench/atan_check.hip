// Device atan2f_exact against the host build of the same source (libm_exact.h).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include <random>
#include "libm_exact.h"
__global__ void k(const float* y, const float* x, float* o, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = lphy_libm::atan2f_exact(y[i], x[i]);
}
int main() {
    const int n = 1 << 22;
    std::vector<float> y(n), x(n), o(n);
    std::mt19937 g(7);
    std::normal_distribution<float> d(0.f, 1.f);
    for (int i = 0; i < n; ++i) { y[i] = d(g) * (i % 7 + 1); x[i] = d(g); }
    float *dy, *dx, *dox;
    hipMalloc(&dy, n * 4); hipMalloc(&dx, n * 4); hipMalloc(&dox, n * 4);
    hipMemcpy(dy, y.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dy, dx, dox, n);
    hipMemcpy(o.data(), dox, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) {
        float h = lphy_libm::atan2f_exact(y[i], x[i]);
        if (memcmp(&h, &o[i], 4)) { if (bad < 5) printf("y=%a x=%a host=%a dev=%a\n", y[i], x[i], h, o[i]); ++bad; }
    }
    printf("atan2 mismatches: %d of %d\n", bad, n);
    return bad != 0;
}
