// Host-side rates of the GPU box that bound the real call path (hc_phmm_pairs_flat):
// pinned allocation cost, H2D / D2H copy rate from pinned memory, and the host's
// multi-threaded copy rate (pageable caller buffers -> pinned staging).
//   hipcc -O2 -std=c++17 -pthread tools/probe_host.cpp -o /tmp/probe_host && /tmp/probe_host
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    const size_t MB = size_t(1) << 20;
    for (size_t sz : {size_t(16) * MB, size_t(64) * MB, size_t(256) * MB}) {
        char* p = nullptr;
        const double t0 = now_ms();
        if (hipHostMalloc(&p, sz, hipHostMallocPortable) != hipSuccess) return 1;
        const double t1 = now_ms();
        (void)hipHostFree(p);
        std::printf("{\"probe\":\"hipHostMalloc\",\"MB\":%zu,\"ms\":%.3f}\n", sz / MB, t1 - t0);
    }
    const size_t N = size_t(512) * MB;
    char *h = nullptr, *d = nullptr;
    if (hipHostMalloc(&h, N, hipHostMallocPortable) != hipSuccess || hipMalloc(&d, N) != hipSuccess) return 1;
    std::memset(h, 1, N);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (size_t chunk : {size_t(4) * MB, size_t(16) * MB, size_t(64) * MB, N}) {
        for (int dir = 0; dir < 2; ++dir) {
            (void)hipDeviceSynchronize();
            double best = 1e30;
            for (int rep = 0; rep < 3; ++rep) {
                const double t0 = now_ms();
                for (size_t o = 0; o < N; o += chunk)
                    (void)hipMemcpyAsync(dir ? h + o : d + o, dir ? d + o : h + o, chunk,
                                         dir ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice, s);
                (void)hipStreamSynchronize(s);
                best = std::min(best, now_ms() - t0);
            }
            std::printf("{\"probe\":\"%s\",\"chunk_MB\":%zu,\"GBs\":%.1f}\n", dir ? "D2H" : "H2D", chunk / MB,
                        double(N) / best / 1e6);
        }
    }
    // Host copy rate: pageable source (fresh, touched) -> pinned destination.
    std::vector<char> src(N, 3);
    for (int T : {1, 4, 8, 16}) {
        double best = 1e30;
        for (int rep = 0; rep < 3; ++rep) {
            std::vector<std::thread> th;
            const double t0 = now_ms();
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    const size_t a = N / T * t, e = t + 1 == T ? N : N / T * (t + 1);
                    std::memcpy(h + a, src.data() + a, e - a);
                });
            for (auto& x : th) x.join();
            best = std::min(best, now_ms() - t0);
        }
        std::printf("{\"probe\":\"host_memcpy\",\"threads\":%d,\"GBs\":%.1f}\n", T, double(N) / best / 1e6);
    }
    // Host read rate (sum of bytes), the gap-constancy scan's access pattern.
    for (int T : {1, 8, 16}) {
        double best = 1e30;
        std::vector<unsigned long long> acc(size_t(T) * 8);
        for (int rep = 0; rep < 3; ++rep) {
            std::vector<std::thread> th;
            const double t0 = now_ms();
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    const size_t a = N / T * t, e = t + 1 == T ? N : N / T * (t + 1);
                    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(src.data() + a);
                    unsigned long long x = 0;
                    for (size_t k = 0; k < (e - a) / 8; ++k) x |= q[k] ^ 0x0303030303030303ull;
                    acc[size_t(t) * 8] = x;
                });
            for (auto& x : th) x.join();
            best = std::min(best, now_ms() - t0);
        }
        std::printf("{\"probe\":\"host_read\",\"threads\":%d,\"GBs\":%.1f}\n", T, double(N) / best / 1e6);
    }
    (void)hipFree(d);
    (void)hipHostFree(h);
    return 0;
}
