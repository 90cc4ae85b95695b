// First-launch cost of a code object with and without rocPRIM's device-wide
// scan instantiated in it (WITH_SCAN=1: hipcub::DeviceScan::ExclusiveSum over
// uint64, which instantiates its kernels for every architecture in rocPRIM's
// table).  Prints the times of: the first HIP call, the first launch of a
// trivial kernel of this code object, a second launch.
#include <hip/hip_runtime.h>
#if WITH_SCAN
#include <hipcub/hipcub.hpp>
#endif
#include <chrono>
#include <cstdio>

__global__ void touch(int* p) { if (threadIdx.x == 0) p[0] = 1; }

#if WITH_SCAN
hipError_t scan(void* t, size_t& b, const uint64_t* in, uint64_t* out, int n, hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(t, b, in, out, n, s);
}
#endif

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
    auto t0 = std::chrono::steady_clock::now();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return 1;
    int* p = nullptr;
    if (hipMalloc(&p, 4) != hipSuccess) return 1;
    const double init = ms_since(t0);
    auto t1 = std::chrono::steady_clock::now();
    touch<<<1, 64>>>(p);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    const double first = ms_since(t1);
    auto t2 = std::chrono::steady_clock::now();
    touch<<<1, 64>>>(p);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    const double second = ms_since(t2);
    printf("{\"with_scan\": %d, \"init_ms\": %.2f, \"first_launch_ms\": %.2f, \"second_launch_ms\": %.3f}\n",
           WITH_SCAN, init, first, second);
    (void)hipFree(p);
    return 0;
}
