// rcp_probe.hip — accuracy of v_rcp_f64 and of one / two Newton steps against the IEEE quotient,
// over log-uniform x in [1e-8, 1e8] (gfx950).  Decides how many Newton steps the pivots need.
//   hipcc --offload-arch=gfx950 -O3 tools/rcp_probe.hip -o gpurun_out/rcp_probe && gpurun_out/rcp_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void probe(const double *x, double *out, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double d = x[i];
    double r = __builtin_amdgcn_rcp(d);
    {   // one step of the quadratic correction r (1 + e + e^2), e = 1 - d r
        const double e0 = __builtin_fma(-d, r, 1.0);
        out[3 * i] = __builtin_fma(r, __builtin_fma(e0, e0, e0), r);
    }
    double e = __builtin_fma(-d, r, 1.0);
    const double r1 = __builtin_fma(r, e, r);
    out[3 * i + 1] = r1;
    e = __builtin_fma(-d, r1, 1.0);
    out[3 * i + 2] = __builtin_fma(r1, e, r1);
}

int main()
{
    const int n = 1 << 22;
    double *hx = (double *)malloc(n * sizeof(double)), *ho = (double *)malloc(3 * n * sizeof(double));
    srand(12345);
    for (int i = 0; i < n; i++) {
        const double u = (double)rand() / RAND_MAX, v = (double)rand() / RAND_MAX;
        hx[i] = pow(10.0, -8.0 + 16.0 * u) * (1.0 + v * 1e-3) * ((i & 1) ? 1.0 : -1.0);
    }
    double *dx, *dout;
    hipMalloc(&dx, n * sizeof(double));
    hipMalloc(&dout, 3 * n * sizeof(double));
    hipMemcpy(dx, hx, n * sizeof(double), hipMemcpyHostToDevice);
    probe<<<n / 256, 256>>>(dx, dout, n);
    hipMemcpy(ho, dout, 3 * n * sizeof(double), hipMemcpyDeviceToHost);
    double worst[3] = {0, 0, 0};
    long exact[3] = {0, 0, 0};
    for (int i = 0; i < n; i++) {
        const double ref = 1.0 / hx[i];
        const double ulp = fabs(nextafter(ref, INFINITY) - ref);
        for (int k = 0; k < 3; k++) {
            const double err = fabs(ho[3 * i + k] - ref) / ulp;
            if (err > worst[k]) worst[k] = err;
            if (ho[3 * i + k] == ref) exact[k]++;
        }
    }
    const char *name[3] = {"quadratic", "+1 Newton", "+2 Newton"};
    for (int k = 0; k < 3; k++) printf("%-10s max error %.3g ulp, exact %.4f\n", name[k], worst[k], (double)exact[k] / n);
    return 0;
}
