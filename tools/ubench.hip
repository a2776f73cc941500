// ubench.hip — issue cost / latency of the instructions the rollout kernel is made of, one wave
// on one SIMD (gfx950).  Prints shader cycles per instruction (s_memtime ticks).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench.hip -o gpurun_out/ubench && gpurun_out/ubench
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 256
#define REP8(x) x x x x x x x x

template <int MODE>
__global__ void bench(double *out, long long *cyc, double seed)
{
    double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const double b = 1.0000001, c = 1e-9;
    __shared__ double lds[512];
    lds[threadIdx.x] = a0;
    __syncthreads();
    int addr = (threadIdx.x & 7) * 8;
    int i0 = threadIdx.x, i1 = 1, i2 = 2 + threadIdx.x, i3 = 3;
    typedef double d4 __attribute__((ext_vector_type(4)));
    d4 m0 = {a0, a1, a2, a3}, m1 = m0, m2 = m0, m3 = m0;
    long long t0 = clock64();
    for (int it = 0; it < ITERS; it++) {
        if (MODE == 0) {   // 8 independent f64 FMA chains
            REP8(asm volatile("v_fma_f64 %0, %2, %3, %0\n v_fma_f64 %1, %2, %3, %1\n" : "+v"(a0), "+v"(a1) : "v"(b), "v"(c));
                 asm volatile("v_fma_f64 %0, %2, %3, %0\n v_fma_f64 %1, %2, %3, %1\n" : "+v"(a2), "+v"(a3) : "v"(b), "v"(c));)
        } else if (MODE == 1) {   // one dependent f64 FMA chain
            REP8(asm volatile("v_fma_f64 %0, %1, %2, %0\n v_fma_f64 %0, %1, %2, %0\n" : "+v"(a0) : "v"(b), "v"(c));)
        } else if (MODE == 2) {   // independent f64 add
            REP8(asm volatile("v_add_f64 %0, %0, %2\n v_add_f64 %1, %1, %2\n" : "+v"(a0), "+v"(a1) : "v"(c));)
        } else if (MODE == 3) {   // independent dpp moves (32-bit)
            REP8(asm volatile("v_mov_b32_dpp %0, %2 row_shr:1 bound_ctrl:0\n v_mov_b32_dpp %1, %3 row_shr:1 bound_ctrl:0\n"
                              : "=v"(i0), "=v"(i1) : "v"(i2), "v"(i3));)
            a0 += i0 + i1;
        } else if (MODE == 4) {   // dependent butterfly stage (compiler-generated): x += mov_dpp(x)
            REP8({
                const int lo = __builtin_amdgcn_mov_dpp(__double2loint(a0), 0xB1, 0xF, 0xF, true);
                const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(a0), 0xB1, 0xF, 0xF, true);
                a0 = a0 + __hiloint2double(hi, lo);
                const int lo2 = __builtin_amdgcn_mov_dpp(__double2loint(a0), 0x4E, 0xF, 0xF, true);
                const int hi2 = __builtin_amdgcn_mov_dpp(__double2hiint(a0), 0x4E, 0xF, 0xF, true);
                a0 = a0 + __hiloint2double(hi2, lo2);
            })
        } else if (MODE == 5) {   // f64 add with DPP operand (row_shr) — 64-bit DPP on gfx950?
            REP8(asm volatile("v_mul_f64 %0, %0, %2\n v_mul_f64 %1, %1, %2\n" : "+v"(a0), "+v"(a1) : "v"(b));)
        } else if (MODE == 6) {   // LDS broadcast read b128 (independent)
            double2 v0, v1;
            REP8(asm volatile("ds_read_b128 %0, %2\n ds_read_b128 %1, %2 offset:16\n" : "=v"(v0), "=v"(v1) : "v"(addr));)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            a0 += v0.x + v1.y;
        } else if (MODE == 7) {   // v_rcp_f64 independent
            REP8(asm volatile("v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n" : "+v"(a0), "+v"(a1));)
        } else if (MODE == 9) {   // v_mov_b64
            REP8(asm volatile("v_mov_b64 %0, %2\n v_mov_b64 %1, %3\n" : "=v"(a0), "=v"(a1) : "v"(a2), "v"(a3));)
        } else if (MODE == 10) {   // dependent LDS write -> read round trip
            REP8(asm volatile("ds_write_b64 %1, %0\n s_waitcnt lgkmcnt(0)\n ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)\n" : "+v"(a0) : "v"(addr));)
        } else if (MODE == 12) {   // independent v_fmac_f64_dpp row_newbcast (8 accumulators)
            REP8(asm volatile("v_fmac_f64_dpp %0, %4, %5 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                              "v_fmac_f64_dpp %1, %4, %5 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(b), "v"(c));)
        } else if (MODE == 13) {   // dependent v_fmac_f64_dpp chain
            REP8(asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                              "s_nop 1\n"
                              "v_fmac_f64_dpp %0, %1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                              "s_nop 1\n"
                              : "+v"(a0) : "v"(b), "v"(c));)
        } else if (MODE == 14) {   // independent v_fmac_f64_dpp, 4 accumulators interleaved
            REP8(asm volatile("v_fmac_f64_dpp %0, %4, %5 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                              "v_fmac_f64_dpp %1, %4, %5 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                              "v_fmac_f64_dpp %2, %4, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                              "v_fmac_f64_dpp %3, %4, %5 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(b), "v"(c));)
        } else if (MODE == 15) {   // dependent v_add_f64 chain
            REP8(asm volatile("v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n" : "+v"(a0) : "v"(c));)
        } else if (MODE == 16) {   // independent v_mfma_f64_16x16x4_f64, 4 accumulators (the M = S^T F A/B)
            REP8({
                m0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b, m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b, m1, 0, 0, 0);
                m2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, b, m2, 0, 0, 0);
                m3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a3, b, m3, 0, 0, 0);
            })
        } else if (MODE == 17) {   // dependent v_mfma_f64_16x16x4_f64 chain
            REP8({
                m0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b, m0, 0, 0, 0);
                m0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b, m0, 0, 0, 0);
            })
        } else if (MODE == 18) {   // dependent v_rcp_f64 chain
            REP8(asm volatile("v_rcp_f64 %0, %0\n s_nop 0\n v_rcp_f64 %0, %0\n s_nop 0\n" : "+v"(a0));)
        } else if (MODE == 19) {   // dependent fmac_f64_dpp -> mov_b64_dpp bcast -> rcp -> fma (one pivot's chain)
            REP8(asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n"
                              "v_mov_b64_dpp %0, %0 row_newbcast:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n s_nop 0\n"
                              : "+v"(a0) : "v"(c));)
        } else if (MODE == 11) {   // independent f32 FMA (reference point)
            float f0 = a0, f1 = a1;
            REP8(asm volatile("v_fma_f32 %0, %2, %2, %0\n v_fma_f32 %1, %2, %2, %1\n" : "+v"(f0), "+v"(f1) : "v"((float)c));)
            a0 = f0 + f1;
        }
    }
    long long t1 = clock64();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + m0.x + m1.y + m2.z + m3.w;
}

template <int MODE>
void run(const char *name, int blocks, double *d_out, long long *d_cyc)
{
    hipLaunchKernelGGL(bench<MODE>, dim3(blocks), dim3(64), 0, 0, d_out, d_cyc, 1.0);
    hipDeviceSynchronize();
    long long h[2048];
    hipMemcpy(h, d_cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < blocks; i++) m += h[i];
    m /= blocks;
    const double per = MODE == 0 || MODE == 14 ? 32.0 : (MODE == 16 ? 32.0 : (MODE == 19 ? 8.0 : 16.0));
    printf("%-34s blocks=%5d  cyc/instr = %.2f\n", name, blocks, m / (ITERS * per));
}

int main()
{
    double *d_out;
    long long *d_cyc;
    hipMalloc(&d_out, 2048 * 64 * sizeof(double));
    hipMalloc(&d_cyc, 2048 * sizeof(long long));
    for (int blocks : {1, 1024, 2048}) {
        run<0>("fma_f64 indep", blocks, d_out, d_cyc);
        run<1>("fma_f64 dependent", blocks, d_out, d_cyc);
        run<2>("add_f64 indep", blocks, d_out, d_cyc);
        run<5>("mul_f64 indep", blocks, d_out, d_cyc);
        run<3>("mov_b32_dpp indep", blocks, d_out, d_cyc);
        run<4>("butterfly stage, per stage (x2 per 16)", blocks, d_out, d_cyc);
        run<6>("ds_read_b128 broadcast", blocks, d_out, d_cyc);
        run<7>("rcp_f64 indep", blocks, d_out, d_cyc);
        run<9>("mov_b64 indep", blocks, d_out, d_cyc);
        run<10>("lds write->read roundtrip", blocks, d_out, d_cyc);
        run<11>("fma_f32 indep", blocks, d_out, d_cyc);
        run<12>("fmac_f64_dpp indep (2 acc)", blocks, d_out, d_cyc);
        run<13>("fmac_f64_dpp dependent (+nop1)", blocks, d_out, d_cyc);
        run<14>("fmac_f64_dpp indep (4 acc)", blocks, d_out, d_cyc);
        run<15>("add_f64 dependent", blocks, d_out, d_cyc);
        run<16>("mfma_f64_16x16x4 indep (4 acc)", blocks, d_out, d_cyc);
        run<17>("mfma_f64_16x16x4 dependent", blocks, d_out, d_cyc);
        run<18>("rcp_f64 dependent (+nop0)", blocks, d_out, d_cyc);
        run<19>("fmac_dpp->mov_b64_dpp pair (per pair)", blocks, d_out, d_cyc);
    }
    return 0;
}
