// occupancy_probe.hip — how many 1-wave workgroups does an MI355X keep resident?
// (diagnostic, not part of the product)
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/occ tools/occupancy_probe.hip && /tmp/occ
//
// Every wave records s_memrealtime (100 MHz) at start and end around a fixed
// VALU busy loop; the host reports the launch span and the peak number of
// waves alive at once, for several LDS sizes and waves per workgroup.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

template <int WPB>
__global__ __launch_bounds__(64 * WPB) void probe(unsigned long long *t, int iters, int lds_bytes) {
    extern __shared__ unsigned char smem[];
    const int wv = threadIdx.x >> 6;
    const long e = (long)blockIdx.x * WPB + wv;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    float x = threadIdx.x;
    // iters < 0: mixed workload, 24% of waves run -iters iterations, the rest -iters/10
    int it = iters;
    if (iters < 0) {
        const unsigned h = (unsigned)(e * 2654435761u) >> 16;
        it = (h % 100u) < 24u ? -iters : -iters / 10;
    }
    for (int i = 0; i < it; i++) x = x * 1.0001f + 0.5f;
    if (lds_bytes) smem[threadIdx.x % lds_bytes] = (unsigned char)x;
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        t[2 * e] = t0;
        t[2 * e + 1] = t1 + (x == 12345.f);
    }
}

template <int WPB>
static void run(int n, int iters, int lds) {
    unsigned long long *d;
    (void)hipMalloc(&d, sizeof(unsigned long long) * 2 * n);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(probe<WPB>, dim3(n / WPB), dim3(64 * WPB), lds * WPB, 0, d, iters, lds);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> h(2 * n);
    (void)hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * n, hipMemcpyDeviceToHost);
    std::vector<std::pair<unsigned long long, int>> ev;
    unsigned long long tmin = ~0ULL, tmax = 0;
    double life = 0;
    for (int i = 0; i < n; i++) {
        ev.push_back({h[2 * i], 1});
        ev.push_back({h[2 * i + 1], -1});
        tmin = std::min(tmin, h[2 * i]);
        tmax = std::max(tmax, h[2 * i + 1]);
        life += (double)(h[2 * i + 1] - h[2 * i]);
    }
    std::sort(ev.begin(), ev.end(), [](auto &x, auto &y) { return x.first < y.first || (x.first == y.first && x.second < y.second); });
    int cur = 0, peak = 0;
    for (auto &p : ev) { cur += p.second; peak = std::max(peak, cur); }
    const double span_us = (tmax - tmin) / 100.0;
    printf("WPB=%d lds=%5d iters=%6d n=%d: event %.1f us, wave span %.1f us, mean life %.2f us, peak alive %d (%.1f/CU), mean alive %.0f\n",
           WPB, lds, iters, n, ms * 1e3, span_us, life / n / 100.0, peak, peak / 256.0, life / (tmax - tmin));
    (void)hipFree(d);
}

int main() {
    const int n = 65536;
    run<1>(n, -500, 1856);
    run<1>(n, -1000, 1856);
    run<1>(n, -2000, 1856);
    for (int iters : {0, 200, 2000}) {
        run<1>(n, iters, 0);
        run<1>(n, iters, 1856);
        run<2>(n, iters, 1856);
        run<4>(n, iters, 1856);
    }
    return 0;
}
