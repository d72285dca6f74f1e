// Test program (tests/test_kernels_gpu.py::test_packed_fp32_coresident): the packed-fp32 sequence the SLP
// vectorizer formed in the deformation backward's HexPlane product, in isolation.
//
// hipcc (-O3, SLP on) builds the bilinear weights as broadcast products
//     v_pk_mul_f32 P, W, W op_sel:[0,1] op_sel_hi:[0,1]      ; P = (w.x * w.y, w.x * w.y)
// and uses P in the very next instruction with no wait state:
//     v_pk_mul_f32 R, D, P                                   ; R = (d.x * P.x, d.y * P.y)
// while a plain v_pk_mul_f32 producer always gets one (an independent instruction or s_nop 0).  In the
// deformation backward (256 threads, 70 KB LDS: two blocks per CU) the low halves of such results came
// out wrong in lanes 48..63, run to run.  This program runs the sequence under 1, 2 and 4 blocks per CU
// (dynamic LDS), in four forms, and counts results that differ from the exact float products:
//   mode 0  broadcast producer -> consumer back to back     (the compiler's schedule)
//   mode 1  the same with s_nop 0 between them
//   mode 2  broadcast producer -> consumer with s_nop 1
//   mode 3  scalar v_mul_f32 chain (the -fno-slp-vectorize form)
//   mode 4  the broadcast IN PLACE (destination = source pair, as 19 of the failing build's 48
//           broadcasts are: v_pk_mul_f32 v[n:n+1], v[n:n+1], v[n:n+1] op_sel:[0,1] op_sel_hi:[0,1]),
//           its source pair written by the packed move just before it, then the consumer
//   mode 5  the in-place broadcast on a pair written long before, then the consumer
//   mode 6  the broadcast on a weight pair fresh from a global load, in the top VGPRs (v[240:245]:
//           the kernel then allocates the whole 256-entry budget, as the deformation backward does)
// (round 5: the in-place form is the one only the failing build contains; modes 0-3 never mismatched)
// Every result is a correctly rounded IEEE product or sum, so the expected values are exact on the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

constexpr int ITERS = 48;

template <int MODE>
__global__ void __launch_bounds__(256) k_pk(const float2* __restrict__ w, const float2* __restrict__ d,
                                              float2* __restrict__ out, int n_per) {
    extern __shared__ float s_pad[];   // only sizes the block's LDS (co-residency)
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (threadIdx.x == 1023) s_pad[0] = 0.0f;   // never true: keeps the allocation
    float2 acc = make_float2(0.0f, 0.0f);
    const float2 wv = w[t];
    for (int i = 0; i < n_per; ++i) {
        float2 dv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) dv[j] = d[((size_t)i * 8 + j) * gridDim.x * 256 + t];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float2 r;
            if constexpr (MODE == 0) {
                asm volatile("v_pk_mul_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[0,1]\n\t"
                             "v_pk_mul_f32 %0, %2, %0"
                             : "=&v"(r) : "v"(wv), "v"(dv[j]));
            } else if constexpr (MODE == 1) {
                asm volatile("v_pk_mul_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[0,1]\n\t"
                             "s_nop 0\n\t"
                             "v_pk_mul_f32 %0, %2, %0"
                             : "=&v"(r) : "v"(wv), "v"(dv[j]));
            } else if constexpr (MODE == 2) {
                asm volatile("v_pk_mul_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[0,1]\n\t"
                             "s_nop 1\n\t"
                             "v_pk_mul_f32 %0, %2, %0"
                             : "=&v"(r) : "v"(wv), "v"(dv[j]));
            } else if constexpr (MODE == 4) {
                asm volatile("v_pk_mov_b32 %0, %1, %1 op_sel:[0,1]\n\t"
                             "v_pk_mul_f32 %0, %0, %0 op_sel:[0,1] op_sel_hi:[0,1]\n\t"
                             "v_pk_mul_f32 %0, %2, %0"
                             : "=&v"(r) : "v"(wv), "v"(dv[j]));
            } else if constexpr (MODE == 6) {
                const float2 wj = w[(t + j * 256) % (gridDim.x * 256)];   // a fresh load per product
                asm volatile("v_mov_b32 v240, %1\n\t"
                             "v_mov_b32 v241, %2\n\t"
                             "v_pk_mul_f32 v[242:243], v[240:241], v[240:241] op_sel:[0,1] op_sel_hi:[0,1]\n\t"
                             "v_pk_mul_f32 %0, %3, v[242:243]"
                             : "=&v"(r) : "v"(wj.x), "v"(wj.y), "v"(dv[j])
                             : "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249",
                               "v250", "v251", "v252", "v253", "v254", "v255");
            } else if constexpr (MODE == 5) {
                r = wv;
                asm volatile("v_pk_mul_f32 %0, %0, %0 op_sel:[0,1] op_sel_hi:[0,1]\n\t"
                             "v_pk_mul_f32 %0, %1, %0"
                             : "+v"(r) : "v"(dv[j]));
            } else {
                float p;
                asm volatile("v_mul_f32 %0, %1, %2" : "=v"(p) : "v"(wv.x), "v"(wv.y));
                asm volatile("v_mul_f32 %0, %2, %3\n\tv_mul_f32 %1, %4, %3"
                             : "=&v"(r.x), "=&v"(r.y) : "v"(dv[j].x), "v"(p), "v"(dv[j].y));
            }
            acc.x += r.x;
            acc.y += r.y;
        }
    }
    out[t] = acc;
}

static float bits_rand(unsigned& s) {
    s = s * 1664525u + 1013904223u;
    return 0.5f + (float)(s >> 8) * (1.0f / 16777216.0f);
}

int main(int argc, char** argv) {
    int cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
    const int blocks = cus * 8, T = blocks * 256, n_per = ITERS / 8;
    std::vector<float2> hw(T), hd((size_t)ITERS * T);
    unsigned s = 12345u;
    for (auto& v : hw) v = make_float2(bits_rand(s), bits_rand(s));
    for (auto& v : hd) v = make_float2(bits_rand(s), bits_rand(s));
    std::vector<float2> ref(T), ref6(T);
    for (int t = 0; t < T; ++t) {
        float ax = 0.0f, ay = 0.0f, bx = 0.0f, by = 0.0f;
        const float p = hw[t].x * hw[t].y;
        for (int k = 0; k < ITERS; ++k) {
            const float2 dv = hd[(size_t)k * T + t];
            ax += dv.x * p;
            ay += dv.y * p;
            const float2 wj = hw[(t + (k % 8) * 256) % T];
            const float pj = wj.x * wj.y;
            bx += dv.x * pj;
            by += dv.y * pj;
        }
        ref[t] = make_float2(ax, ay);
        ref6[t] = make_float2(bx, by);
    }
    float2 *dw, *dd, *dout;
    if (hipMalloc(&dw, T * 8) != hipSuccess || hipMalloc(&dd, hd.size() * 8) != hipSuccess ||
        hipMalloc(&dout, T * 8) != hipSuccess) { printf("alloc failed\n"); return 2; }
    (void)hipMemcpy(dw, hw.data(), T * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dd, hd.data(), hd.size() * 8, hipMemcpyHostToDevice);
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const size_t lds_for[3] = {100 * 1024, 70 * 1024, 36 * 1024};   // 1, 2, 4 blocks per CU
    const char* names[7] = {"broadcast->consumer back to back", "broadcast, s_nop 0, consumer",
                            "broadcast, s_nop 1, consumer", "scalar v_mul_f32",
                            "pk_mov -> in-place broadcast -> consumer", "in-place broadcast -> consumer",
                            "fresh-load broadcast in v[240:243] -> consumer"};
    int total_bad = 0, bad_modes[7] = {0, 0, 0, 0, 0, 0, 0};
    std::vector<float2> o(T);
    for (int mode = 0; mode < 7; ++mode) {
        for (int li = 0; li < 3; ++li) {
            long bad = 0, bad_lo = 0, bad_hi = 0, by_quarter[4] = {0, 0, 0, 0};
            for (int r = 0; r < reps; ++r) {
                (void)hipMemset(dout, 0xFF, T * 8);
                auto kern = mode == 0 ? k_pk<0> : mode == 1 ? k_pk<1> : mode == 2 ? k_pk<2> : mode == 3 ? k_pk<3>
                          : mode == 4 ? k_pk<4> : mode == 5 ? k_pk<5> : k_pk<6>;
                hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds_for[li], 0, dw, dd, dout, n_per);
                if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
                (void)hipMemcpy(o.data(), dout, T * 8, hipMemcpyDeviceToHost);
                const std::vector<float2>& rf = mode == 6 ? ref6 : ref;
                for (int t = 0; t < T; ++t) {
                    const bool lo = memcmp(&o[t].x, &rf[t].x, 4) != 0, hi = memcmp(&o[t].y, &rf[t].y, 4) != 0;
                    if (lo || hi) {
                        ++bad; bad_lo += lo; bad_hi += hi;
                        ++by_quarter[(t & 63) >> 4];
                    }
                }
            }
            printf("mode %d (%s), %d block(s)/CU: %ld wrong of %ld (low %ld, high %ld; lanes 0-15/16-31/32-47/48-63: "
                   "%ld/%ld/%ld/%ld)\n", mode, names[mode], li == 0 ? 1 : (li == 1 ? 2 : 4), bad, (long)T * reps,
                   bad_lo, bad_hi, by_quarter[0], by_quarter[1], by_quarter[2], by_quarter[3]);
            bad_modes[mode] += (int)(bad > 0);
            total_bad += (int)(bad > 0);
        }
    }
    printf("packed fp32 co-residency: %s\n", total_bad ? "MISMATCHES" : "ok");
    // the exit status reports the forms the build uses: the scalar chain (mode 3) and the nop-separated
    // packed forms must be exact; modes 0, 4, 5 and 6 are the reproducer candidates and only reported
    return (bad_modes[1] || bad_modes[2] || bad_modes[3]) ? 1 : 0;
}
