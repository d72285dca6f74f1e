// The -amdgpu-waitcnt-forcezero fault: that debug flag inserts an
// "s_waitcnt vmcnt(0) expcnt(0) lgkmcnt(0)" before nearly every instruction, and the hazard recognizer
// then counts each of them as one wait state and drops the s_nop it had placed for a hazard.  In the
// deformation build the dropped nops guard (among others) "VALU writes VCC -> v_cndmask reads VCC" in
// the unsigned-division fix-up of k_pack_weight, whose quotient is a row index.  This kernel runs that
// exact instruction pattern on data: 32-bit unsigned division / remainder by a kernel argument (the
// quotient fix-ups are v_cmp -> v_cndmask pairs) and a correctly rounded sqrt (v_cmp_class -> v_cndmask),
// and stores the results (no data-dependent addressing, so a wrong value cannot fault).
//   t_waitcnt_hazard            exit 0 iff every result equals the host's
// Built twice by tests/test_kernels_gpu.py: as the library is built, and with the debug flag.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_div(const unsigned* __restrict__ a, unsigned d, unsigned* __restrict__ q, unsigned* __restrict__ r,
                      const float* __restrict__ x, float* __restrict__ s, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned v = a[i];
    q[i] = v / d;
    r[i] = v % d;
    s[i] = sqrtf(x[i]);
}

int main() {
    const int n = 1 << 22;
    std::vector<unsigned> a(n);
    std::vector<float> x(n);
    unsigned long long st = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        a[i] = (unsigned)st;
        x[i] = (float)((st >> 40) & 0xFFFFFF) * 0.37f + 1e-3f;
    }
    unsigned *da, *dq, *dr;
    float *dx, *ds;
    hipMalloc(&da, n * 4); hipMalloc(&dq, n * 4); hipMalloc(&dr, n * 4); hipMalloc(&dx, n * 4); hipMalloc(&ds, n * 4);
    hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    std::vector<unsigned> q(n), r(n);
    std::vector<float> s(n);
    long bad_q = 0, bad_s = 0;
    const unsigned divs[] = {3u, 7u, 48u, 128u, 1000u, 4096u, 65537u, 2147483659u};
    for (unsigned d : divs) {
        hipLaunchKernelGGL(k_div, dim3((n + 255) / 256), dim3(256), 0, 0, da, d, dq, dr, dx, ds, n);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
        hipMemcpy(q.data(), dq, n * 4, hipMemcpyDeviceToHost);
        hipMemcpy(r.data(), dr, n * 4, hipMemcpyDeviceToHost);
        hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
        long bq = 0, bs = 0;
        for (int i = 0; i < n; ++i) {
            if (q[i] != a[i] / d || r[i] != a[i] % d) ++bq;
            if (s[i] != std::sqrt(x[i])) ++bs;
        }
        printf("d=%u: %ld wrong quotients/remainders, %ld wrong sqrt of %d\n", d, bq, bs, n);
        bad_q += bq;
        bad_s += bs;
    }
    printf("total wrong: div %ld, sqrt %ld\n", bad_q, bad_s);
    return (bad_q || bad_s) ? 1 : 0;
}
