// hbm_write_probe.hip - achievable HBM store bandwidth on this box for the point-cloud kernel's pattern:
// 16-B stores per lane, plain vs non-temporal, one workgroup per 10.7 KB "env" chunk vs a flat grid.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/hbm_write_probe tools/probes/hbm_write_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void __launch_bounds__(256) flat_store(f4* out, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    f4 v = {(float)i, 1.f, 2.f, 3.f};
    if (NT) __builtin_nontemporal_store(v, out + i);
    else out[i] = v;
}

template <bool NT>
__global__ void __launch_bounds__(256) env_store(f4* out, int W) {
    f4* o = out + (size_t)blockIdx.x * W;
    for (int i = threadIdx.x; i < W; i += 256) {
        f4 v = {(float)i, 1.f, 2.f, 3.f};
        if (NT) __builtin_nontemporal_store(v, o + i);
        else o[i] = v;
    }
}

int main() {
    const int W = 670;                 // points per env (student list)
    for (int N : {8192, 65536}) {
        size_t n = (size_t)N * W;
        f4* d;
        hipMalloc(&d, n * sizeof(f4));
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        for (int v = 0; v < 4; v++) {
            auto run = [&]() {
                if (v == 0) flat_store<false><<<(n + 255) / 256, 256>>>(d, n);
                if (v == 1) flat_store<true><<<(n + 255) / 256, 256>>>(d, n);
                if (v == 2) env_store<false><<<N, 256>>>(d, W);
                if (v == 3) env_store<true><<<N, 256>>>(d, W);
            };
            for (int k = 0; k < 5; k++) run();
            hipEventRecord(a);
            const int it = 50;
            for (int k = 0; k < it; k++) run();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            ms /= it;
            const char* nm[] = {"flat plain", "flat nt", "env-block plain", "env-block nt"};
            printf("N %6d %-16s %8.1f us  %6.0f GB/s\n", N, nm[v], ms * 1e3, n * 16.0 / (ms * 1e-3) / 1e9);
        }
        hipFree(d);
    }
    return 0;
}
