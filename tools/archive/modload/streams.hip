// First use of new HIP streams in a process: after the default stream's first
// launch, streams 1..6 are created one by one and each runs one small H2D copy
// and one trivial kernel; prints each stream's creation and first-use times
// (GPU_MAX_HW_QUEUES hardware queues are shared round-robin by the streams).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void touch(int* p) { if (threadIdx.x == 0) p[0] += 1; }

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
    int* d = nullptr;
    int* h = nullptr;
    if (hipMalloc(&d, 4096) != hipSuccess || hipHostMalloc(&h, 4096, 0) != hipSuccess) return 1;
    auto t = std::chrono::steady_clock::now();
    touch<<<1, 64>>>(d);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("{\"default_first_launch_ms\": %.2f, \"streams\": [", ms_since(t));
    for (int i = 0; i < 6; ++i) {
        hipStream_t s;
        t = std::chrono::steady_clock::now();
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
        const double create = ms_since(t);
        t = std::chrono::steady_clock::now();
        if (hipMemcpyAsync(d, h, 4096, hipMemcpyHostToDevice, s) != hipSuccess) return 1;
        if (hipStreamSynchronize(s) != hipSuccess) return 1;
        const double copy = ms_since(t);
        t = std::chrono::steady_clock::now();
        touch<<<1, 64, 0, s>>>(d);
        if (hipStreamSynchronize(s) != hipSuccess) return 1;
        const double kern = ms_since(t);
        printf("%s{\"create_ms\": %.2f, \"first_copy_ms\": %.2f, \"first_kernel_ms\": %.2f}", i ? ", " : "", create,
               copy, kern);
    }
    printf("]}\n");
    return 0;
}
