// Lab (not shipped): where the fixed HIP start-up cost of a short CLI run goes.
// Times each first-call step of a bare HIP program; with an argument it then
// creates an ek_ctx through the product library (code objects of every
// kernel) so the two can be compared.
// Build: make -C tools; run: tools/build/init_lab [lib]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#include "../include/eigkl.h"

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); }

int main(int argc, char**) {
    auto t0 = clk::now(), t = t0;
    int n = 0;
    (void)hipInit(0);
    std::printf("hipInit            %8.2f ms\n", ms(t));
    t = clk::now();
    (void)hipGetDeviceCount(&n);
    std::printf("hipGetDeviceCount  %8.2f ms (%d devices)\n", ms(t), n);
    t = clk::now();
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    std::printf("getDeviceProps     %8.2f ms (%s)\n", ms(t), p.gcnArchName);
    t = clk::now();
    (void)hipSetDevice(0);
    (void)hipFree(nullptr);
    std::printf("setDevice+free(0)  %8.2f ms\n", ms(t));
    t = clk::now();
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    std::printf("streamCreate       %8.2f ms\n", ms(t));
    t = clk::now();
    void* d = nullptr;
    (void)hipMalloc(&d, 64 << 20);
    std::printf("hipMalloc 64MB     %8.2f ms\n", ms(t));
    if (argc > 1) {
        t = clk::now();
        ek_ctx* c = nullptr;
        const int rc = ek_init(0, &c);
        std::printf("ek_init            %8.2f ms (rc %d)\n", ms(t), rc);
        t = clk::now();
        const int32_t rp[2] = {0, 1}, cl[1] = {0};
        const double v[1] = {1.0};
        double x = 1.0, y = 0.0;
        ek_spmv_setup(c, 1, 0, 1, rp, cl, v);
        ek_spmv_host(c, &x, &y);
        std::printf("first SpMV (load)  %8.2f ms (y %g)\n", ms(t), y);
        ek_destroy(c);
    }
    std::printf("total              %8.2f ms\n", ms(t0));
    return 0;
}
