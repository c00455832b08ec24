// Dev probe: host->device copy rates on this box: pageable (hipMemcpyAsync from malloc'd memory),
// pinned (hipHostMalloc), and pageable -> pinned staging with T host threads feeding a DMA ring.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
    const size_t B = 256ull << 20;
    char* h = (char*)malloc(B);
    memset(h, 1, B);
    char *pin, *d;
    CK(hipHostMalloc((void**)&pin, B, hipHostMallocDefault));
    memset(pin, 2, B);
    CK(hipMalloc((void**)&d, B));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int rep = 0; rep < 3; rep++) {
        double t0 = now();
        CK(hipMemcpyAsync(d, h, B, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        double t1 = now();
        CK(hipMemcpyAsync(d, pin, B, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        double t2 = now();
        printf("pageable %.1f GB/s  pinned %.1f GB/s\n", B / (t1 - t0) / 1e9, B / (t2 - t1) / 1e9);
    }
    // host memcpy into pinned with T threads, then one DMA (no overlap) and a chunked ring (overlap)
    for (int T : {1, 4, 8, 16}) {
        double t0 = now();
        std::vector<std::thread> th;
        for (int i = 0; i < T; i++) th.emplace_back([=] { memcpy(pin + B / T * i, h + B / T * i, B / T); });
        for (auto& x : th) x.join();
        double t1 = now();
        printf("memcpy to pinned, %d threads: %.1f GB/s\n", T, B / (t1 - t0) / 1e9);
    }
    const size_t CH = 16ull << 20;
    for (int T : {4, 8}) {
        hipEvent_t ev[4];
        for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        double t0 = now();
        for (size_t off = 0, k = 0; off < B; off += CH, k++) {
            char* slot = pin + (k % 4) * CH;
            if (k >= 4) CK(hipEventSynchronize(ev[k % 4]));
            std::vector<std::thread> th;
            for (int i = 0; i < T; i++) th.emplace_back([=] { memcpy(slot + CH / T * i, h + off + CH / T * i, CH / T); });
            for (auto& x : th) x.join();
            CK(hipMemcpyAsync(d + off, slot, CH, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(ev[k % 4], s));
        }
        CK(hipStreamSynchronize(s));
        double t1 = now();
        printf("ring (16 MB chunks, %d threads per chunk): %.1f GB/s\n", T, B / (t1 - t0) / 1e9);
    }
    return 0;
}
