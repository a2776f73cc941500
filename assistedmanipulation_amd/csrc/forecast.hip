// forecast.hip — the end-effector wrench forecast on the device.
//
// The rollout's trajectory cost asks the forecast for the wrench at t0 + k dt at every step k
// (DynamicsForecast::get_end_effector_wrench, dynamics.hpp:275-278, from
// AssistedManipulation::trajectory_cost, assisted_manipulation.cpp:237-290).  Those values are a
// pure function of t during an update, so each update samples them once into the per-step
// constants the rollout kernel reads:
//
//   forecast_steps_kernel   StepConst[k] for k < H from Forecast::forecast(t0 + k dt): LOCF
//                           (forecast.hpp:109-114), Average (forecast.cpp:124-128) or Kalman
//                           (forecast.cpp:342-367: linear interpolation of the prediction table);
//   kalman_observe_kernel   KalmanForecast::update(measurement, time) (forecast.cpp:298-331): the
//                           deferred update(time) predictions (kalman.cpp:138-152), derivative
//                           estimates, KalmanFilter::update (kalman.cpp:103-136: gain by a
//                           Gauss-Jordan inverse with partial pivoting), and the horison of
//                           predictions F^i x, i <= steps.  One workgroup, matrices in LDS
//                           (n = 6 (order + 1) <= 24 states);
//   forecast_eval_kernel    Forecast::forecast(t) for the host (mppi_forecast_get).

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "engine_types.hpp"
#include "kernels.hpp"

using namespace mppi_eng;

namespace {

constexpr int KT = 256;

__device__ __forceinline__ void forecast_eval(const ForecastArgs &f, double time, double *out)
{
    if (f.type == FC_LOCF) {
        const bool valid = !(time > f.valid_until);
        for (int k = 0; k < 6; k++) out[k] = valid ? f.value[k] : 0.0;
    } else if (f.type == FC_AVERAGE) {
        for (int k = 0; k < 6; k++) out[k] = f.value[k];
    } else if (f.type == FC_KALMAN) {
        if (time > f.last_update + f.horison) {
            for (int k = 0; k < 6; k++) out[k] = 0.0;
            return;
        }
        double t = (time - f.last_update) / f.time_step;
        int lower = (int)t;
        t -= lower;
        // the reference reads column steps + 1 at time == last + horison (out of range): clamped
        lower = lower < 0 ? 0 : (lower > f.steps ? f.steps : lower);
        const int upper = lower + 1 > f.steps ? f.steps : lower + 1;
        for (int k = 0; k < 6; k++) out[k] = (1.0 - t) * f.pred[lower * 6 + k] + t * f.pred[upper * 6 + k];
    } else {
        for (int k = 0; k < 6; k++) out[k] = 0.0;
    }
}

// StepConst of build_steps (engine.cpp) from the forecast: trajectory_cost's per-step terms.
__global__ __launch_bounds__(64) void forecast_steps_kernel(ForecastArgs f, StepParams p, const double *__restrict__ gamma, int H,
                                                            double t0, double dt, StepConst *__restrict__ out)
{
    const int k = blockIdx.x * 64 + threadIdx.x;
    if (k >= H) return;
    StepConst s{};
    s.gamma_k = gamma[k];
    if (p.assisted_manipulation) {
        double F[6];
        // m_rollout_time + step * m_time_step (mppi.cpp:326), rounded twice like the reference: a
        // contracted fma moves times across the forecast's horison cutoff and grid points
        double tk;
        {
#pragma clang fp contract(off)
            tk = t0 + (double)k * dt;
        }
        forecast_eval(f, tk, F);
        for (int i = 0; i < 3; i++) {
            double t = p.target_scale * F[i];
            t = (p.target_maximum < t) ? p.target_maximum : t;   // cwiseMin(max)
            t = (t < -p.target_maximum) ? -p.target_maximum : t; // cwiseMax(-max)
            s.target[i] = t;
        }
        s.tt = (s.target[0] * s.target[0] + s.target[1] * s.target[1]) + s.target[2] * s.target[2];
        const double distance = sqrt(s.tt);
        s.active = (p.has_forecast && distance > p.position_threshold) ? 1 : 0;
        s.pos_cost = (p.pos_c + p.pos_l * fabs(distance)) + p.pos_q * distance * distance;
        double vt = exp(p.vel_dropoff * distance) - 1;
        vt = (vt < p.vel_minimum) ? p.vel_minimum : ((p.vel_maximum < vt) ? p.vel_maximum : vt);
        s.vtarget = vt;
    }
    out[k] = s;
}

// forecast(t0 + k dt), k < steps (DynamicsForecast::forecast's wrench rows, dynamics.cpp:113-123:
// time + step * time_step, two roundings)
__global__ __launch_bounds__(64) void forecast_table_kernel(ForecastArgs f, double t0, double dt, int64_t steps, double *__restrict__ out)
{
    const int64_t k = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (k >= steps) return;
    double tk;
    {
#pragma clang fp contract(off)
        tk = t0 + (double)k * dt;
    }
    forecast_eval(f, tk, out + k * 6);
}

__global__ void forecast_eval_kernel(ForecastArgs f, double time, double *out)
{
    if (threadIdx.x == 0) forecast_eval(f, time, out);
}

// LDS matrix helpers over the whole block (n x n, row-major, stride KMAX)
__device__ __forceinline__ void mat_mul(const double *A, const double *B, double *C, int n, bool transpose_b)
{
    for (int e = threadIdx.x; e < n * n; e += KT) {
        const int i = e / n, j = e % n;
        double s = 0.0;
        for (int l = 0; l < n; l++) s += A[i * KMAX + l] * (transpose_b ? B[j * KMAX + l] : B[l * KMAX + j]);
        C[i * KMAX + j] = s;
    }
}
__device__ __forceinline__ void mat_vec(const double *A, const double *v, double *o, int n)
{
    if ((int)threadIdx.x < n) {
        const int i = threadIdx.x;
        double s = 0.0;
        for (int l = 0; l < n; l++) s += A[i * KMAX + l] * v[l];
        o[i] = s;
    }
}

// P <- F P F^T + Q (Q = 1e-8 I, forecast.cpp:287-296)
__device__ __forceinline__ void propagate(const double *F, double *P, double *T, int n)
{
    mat_mul(F, P, T, n, false);
    __syncthreads();
    mat_mul(T, F, P, n, true);
    __syncthreads();
    if ((int)threadIdx.x < n) P[threadIdx.x * KMAX + threadIdx.x] += 1e-8;
    __syncthreads();
}

__global__ __launch_bounds__(KT) void kalman_observe_kernel(DevKalman *__restrict__ kf, double *__restrict__ pred, KalmanObserve a)
{
    __shared__ double F[KMAX * KMAX], P[KMAX * KMAX], T[KMAX * KMAX], K[KMAX * KMAX];
    __shared__ double G[KMAX * 2 * KMAX];   // [S | I] -> [I | S^-1]
    __shared__ double x[KMAX], xn[KMAX], meas[KMAX], v[KMAX], w[KMAX], fac[KMAX];
    __shared__ double pinv;
    __shared__ int piv;
    const int n = a.n, t = threadIdx.x;
    for (int e = t; e < KMAX * KMAX; e += KT) {
        F[e] = kf->F[e];
        P[e] = kf->P[e];
    }
    if (t < KMAX) {
        x[t] = kf->x[t];
        xn[t] = kf->xn[t];
        meas[t] = kf->meas[t];
    }
    __syncthreads();
    // update(time) calls since the last observation: KalmanFilter::predict()
    for (int64_t r = 0; r < a.pending; r++) {
        if (t < n) x[t] = xn[t];
        __syncthreads();
        mat_vec(F, x, xn, n);
        __syncthreads();
        propagate(F, P, T, n);
    }
    // wrench derivatives (forecast.cpp:304-317)
    if (t < 6) {
        double delta = (a.m[t] - meas[t]) / a.dt;
        for (int i = 1; i <= a.order; i++) {
            const double next = (delta - meas[6 * i + t]) / a.dt;
            meas[6 * i + t] = delta;
            delta = next;
        }
        meas[t] = a.m[t];
    }
    // KalmanFilter::update: S = P + R, gain P S^-1 (H = I, R = 1e-8 I)
    for (int e = t; e < n * 2 * n; e += KT) {
        const int i = e / (2 * n), j = e % (2 * n);
        G[i * 2 * KMAX + j] = (j < n) ? P[i * KMAX + j] + (i == j ? 1e-8 : 0.0) : ((j - n == i) ? 1.0 : 0.0);
    }
    __syncthreads();
    for (int c = 0; c < n; c++) {
        if (t == 0) {
            int p = c;
            for (int r = c + 1; r < n; r++)
                if (fabs(G[r * 2 * KMAX + c]) > fabs(G[p * 2 * KMAX + c])) p = r;
            piv = p;
        }
        __syncthreads();
        if (piv != c)
            for (int j = t; j < 2 * n; j += KT) {
                const double tmp = G[c * 2 * KMAX + j];
                G[c * 2 * KMAX + j] = G[piv * 2 * KMAX + j];
                G[piv * 2 * KMAX + j] = tmp;
            }
        __syncthreads();
        if (t == 0) pinv = 1.0 / G[c * 2 * KMAX + c];
        __syncthreads();
        for (int j = t; j < 2 * n; j += KT) G[c * 2 * KMAX + j] *= pinv;
        if (t < n) fac[t] = G[t * 2 * KMAX + c];
        __syncthreads();
        for (int e = t; e < n * 2 * n; e += KT) {
            const int i = e / (2 * n), j = e % (2 * n);
            if (i != c) G[i * 2 * KMAX + j] -= fac[i] * G[c * 2 * KMAX + j];
        }
        __syncthreads();
    }
    for (int e = t; e < n * n; e += KT) T[(e / n) * KMAX + e % n] = G[(e / n) * 2 * KMAX + n + e % n];
    __syncthreads();
    mat_mul(P, T, K, n, false);   // (P H^T) (H P H^T + R)^-1
    __syncthreads();
    if (t < n) v[t] = meas[t] - xn[t];
    __syncthreads();
    mat_vec(K, v, w, n);
    __syncthreads();
    if (t < n) x[t] = xn[t] + w[t];
    // P <- (I - K H) P
    for (int e = t; e < n * n; e += KT) {
        const int i = e / n, j = e % n;
        double s = 0.0;
        for (int l = 0; l < n; l++) s += ((i == l ? 1.0 : 0.0) - K[i * KMAX + l]) * P[l * KMAX + j];
        T[i * KMAX + j] = s;
    }
    __syncthreads();
    for (int e = t; e < n * n; e += KT) P[(e / n) * KMAX + e % n] = T[(e / n) * KMAX + e % n];
    __syncthreads();
    mat_vec(F, x, xn, n);
    __syncthreads();
    propagate(F, P, T, n);
    // the predictor: F^i x, i <= steps (predict(false) from set_estimation(x))
    if (t < n) v[t] = x[t];
    if (t < 6) pred[t] = x[t];
    __syncthreads();
    for (int s = 0; s < a.steps; s++) {
        double *src = (s & 1) ? w : v, *dst = (s & 1) ? v : w;
        mat_vec(F, src, dst, n);
        __syncthreads();
        if (t < 6) pred[(s + 1) * 6 + t] = dst[t];
    }
    for (int e = t; e < KMAX * KMAX; e += KT) kf->P[e] = P[e];
    if (t < KMAX) {
        kf->x[t] = x[t];
        kf->xn[t] = xn[t];
        kf->meas[t] = meas[t];
    }
}

}  // namespace

namespace mppi_eng {

hipError_t launch_forecast_steps(const ForecastArgs &f, const StepParams &p, const double *gamma, int H, double t0, double dt,
                                 StepConst *out, hipStream_t s)
{
    hipLaunchKernelGGL(forecast_steps_kernel, dim3((H + 63) / 64), dim3(64), 0, s, f, p, gamma, H, t0, dt, out);
    return hipGetLastError();
}

hipError_t launch_kalman_observe(DevKalman *kf, double *pred, const KalmanObserve &a, hipStream_t s)
{
    hipLaunchKernelGGL(kalman_observe_kernel, dim3(1), dim3(KT), 0, s, kf, pred, a);
    return hipGetLastError();
}

hipError_t launch_forecast_table(const ForecastArgs &f, double t0, double dt, int64_t steps, double *out, hipStream_t s)
{
    if (steps <= 0) return hipSuccess;
    hipLaunchKernelGGL(forecast_table_kernel, dim3((unsigned)((steps + 63) / 64)), dim3(64), 0, s, f, t0, dt, steps, out);
    return hipGetLastError();
}

hipError_t launch_forecast_eval(const ForecastArgs &f, double time, double *out, hipStream_t s)
{
    hipLaunchKernelGGL(forecast_eval_kernel, dim3(1), dim3(64), 0, s, f, time, out);
    return hipGetLastError();
}

}  // namespace mppi_eng
