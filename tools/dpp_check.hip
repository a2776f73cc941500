// dpp_check.hip — checks the inline-asm v_fmac_f64_dpp helpers of fr_coop.hip against plain
// shuffles on the GPU.  hipcc --offload-arch=gfx950 -O3 tools/dpp_check.hip -o /tmp/dpp_check
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>

__device__ __forceinline__ double bfma6(double x, const double *y, double acc)
{
    asm("s_nop 1\n\t"
        "v_fmac_f64_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %4 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %6 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, %1, %7 row_newbcast:5 row_mask:0xf bank_mask:0xf"
        : "+v"(acc)
        : "v"(x), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]), "v"(y[4]), "v"(y[5]));
    return acc;
}
__device__ __forceinline__ void bfma6_rank1(double x, double y, double *c)
{
    asm("s_nop 1\n\t"
        "v_fmac_f64_dpp %0, %6, %7 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, %6, %7 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, %6, %7 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, %6, %7 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %4, %6, %7 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %5, %6, %7 row_newbcast:5 row_mask:0xf bank_mask:0xf"
        : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5])
        : "v"(x), "v"(y));
}

__global__ void k(const double *in, double *out)
{
    const int l = threadIdx.x, row = l & ~15;
    const double x = in[l];
    double y[6];
    for (int i = 0; i < 6; i++) y[i] = in[64 + l * 6 + i];
    // reference: sum_r x[row + r] * y[r]
    double ref = 0.0;
    for (int r = 0; r < 6; r++) ref = fma(__shfl(x, row + r, 64), y[r], ref);
    const double got = bfma6(x, y, 0.0);
    double c[6], cref[6];
    for (int i = 0; i < 6; i++) { c[i] = y[i]; cref[i] = fma(__shfl(x, row + i, 64), -x, y[i]); }
    bfma6_rank1(x, -x, c);
    double err = fabs(got - ref);
    for (int i = 0; i < 6; i++) err = fmax(err, fabs(c[i] - cref[i]));
    out[l] = err;
}

int main()
{
    double h[64 + 64 * 6], *din, *dout, e[64];
    for (int i = 0; i < 64 + 64 * 6; i++) h[i] = sin(0.37 * i + 0.1) * (1 + i % 7);
    hipMalloc(&din, sizeof(h));
    hipMalloc(&dout, sizeof(e));
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout);
    hipMemcpy(e, dout, sizeof(e), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 64; i++) m = fmax(m, e[i]);
    printf("dpp helpers max abs err %.3e (%s)\n", m, m < 1e-12 ? "ok" : "MISMATCH");
    return m < 1e-12 ? 0 : 1;
}
