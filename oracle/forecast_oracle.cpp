// forecast_oracle.cpp — TEST INFRASTRUCTURE ONLY (see mppi_oracle.cpp's header): never linked
// into or called by the product.
//
// fp64 restatement of the reference's wrench forecasts (LuigiVan01/AssistedManipulation
// @ 2025-02-05, paths relative to its src/):
//
//   controller/forecast.cpp:6-39     Forecast::create
//   controller/forecast.hpp:64-140   LOCFForecast
//   controller/forecast.cpp:41-129   AverageForecast (create, clear_old_measurements,
//                                    update_average, update, forecast)
//   controller/forecast.cpp:131-367  KalmanForecast (create, transition matrix, update,
//                                    update(time), forecast)
//   controller/kalman.cpp:7-152      KalmanFilter (create, update, predict)
//
// Eigen is absent here: matrices are row-major std::vectors and the inverse in
// KalmanFilter::update is an LU with partial pivoting (what Eigen's MatrixXd::inverse() uses
// for dynamic sizes), so results agree with the reference to rounding, not bit for bit.
// Documented choices where the reference is undefined:
//   * m_prediction is uninitialised until the first observation (forecast.cpp:186): zeros here;
//   * forecast() reads column lower + 1 = steps + 1 at time == last + horison (out of range):
//     the column index is clamped to steps (its weight is then t - lower, usually 0).

#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../include/mppi_amd.h"

namespace {

using Mat = std::vector<double>;   // row-major n x m

Mat matmul(const Mat &A, const Mat &B, int n, int k, int m)
{
    Mat C((size_t)n * m, 0.0);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < m; j++) {
            double s = 0.0;
            for (int l = 0; l < k; l++) s += A[(size_t)i * k + l] * B[(size_t)l * m + j];
            C[(size_t)i * m + j] = s;
        }
    return C;
}

Mat transpose(const Mat &A, int n, int m)
{
    Mat T((size_t)m * n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < m; j++) T[(size_t)j * n + i] = A[(size_t)i * m + j];
    return T;
}

// inverse by LU with partial pivoting (PartialPivLU::inverse)
Mat inverse(const Mat &A0, int n)
{
    Mat A = A0;
    std::vector<int> perm(n);
    for (int i = 0; i < n; i++) perm[i] = i;
    for (int k = 0; k < n; k++) {
        int p = k;
        for (int i = k + 1; i < n; i++)
            if (std::fabs(A[(size_t)i * n + k]) > std::fabs(A[(size_t)p * n + k])) p = i;
        if (p != k) {
            for (int j = 0; j < n; j++) std::swap(A[(size_t)k * n + j], A[(size_t)p * n + j]);
            std::swap(perm[k], perm[p]);
        }
        for (int i = k + 1; i < n; i++) {
            A[(size_t)i * n + k] /= A[(size_t)k * n + k];
            for (int j = k + 1; j < n; j++) A[(size_t)i * n + j] -= A[(size_t)i * n + k] * A[(size_t)k * n + j];
        }
    }
    Mat X((size_t)n * n, 0.0);
    for (int c = 0; c < n; c++) {
        std::vector<double> y(n);
        for (int i = 0; i < n; i++) {   // L y = P e_c
            double s = (perm[i] == c) ? 1.0 : 0.0;
            for (int j = 0; j < i; j++) s -= A[(size_t)i * n + j] * y[j];
            y[i] = s;
        }
        for (int i = n - 1; i >= 0; i--) {   // U x = y
            double s = y[i];
            for (int j = i + 1; j < n; j++) s -= A[(size_t)i * n + j] * X[(size_t)j * n + c];
            X[(size_t)i * n + c] = s / A[(size_t)i * n + i];
        }
    }
    return X;
}

struct KalmanFilter {   // kalman.cpp, H = I, observed_states = states
    int n = 0;
    Mat F, Q, R, P;
    std::vector<double> x, xn;

    std::vector<double> mul(const Mat &M, const std::vector<double> &v) const
    {
        std::vector<double> o(n, 0.0);
        for (int i = 0; i < n; i++) {
            double s = 0.0;
            for (int j = 0; j < n; j++) s += M[(size_t)i * n + j] * v[j];
            o[i] = s;
        }
        return o;
    }
    void propagate_covariance()   // F P F^T + Q
    {
        Mat FP = matmul(F, P, n, n, n);
        P = matmul(FP, transpose(F, n, n), n, n, n);
        for (size_t i = 0; i < P.size(); i++) P[i] += Q[i];
    }
    void update(const std::vector<double> &obs)   // KalmanFilter::update (kalman.cpp:103-136)
    {
        Mat S = P;
        for (size_t i = 0; i < S.size(); i++) S[i] += R[i];
        Mat K = matmul(P, inverse(S, n), n, n, n);
        std::vector<double> innov(n);
        for (int i = 0; i < n; i++) innov[i] = obs[i] - xn[i];
        std::vector<double> Ki = mul(K, innov);
        for (int i = 0; i < n; i++) x[i] = xn[i] + Ki[i];
        Mat IK((size_t)n * n);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) IK[(size_t)i * n + j] = (i == j ? 1.0 : 0.0) - K[(size_t)i * n + j];
        P = matmul(IK, P, n, n, n);
        xn = mul(F, x);
        propagate_covariance();
    }
    void predict(bool cov)   // KalmanFilter::predict (kalman.cpp:138-152)
    {
        x = xn;
        xn = mul(F, x);
        if (cov) propagate_covariance();
    }
};

unsigned factorial(unsigned k) { return k <= 1 ? 1 : k * factorial(k - 1); }

struct OForecast {
    int type = 0;
    // LOCF
    double horison = 0.0, valid_until = 0.0;
    std::vector<double> observation;
    // AVERAGE
    double window = 0.0, last = 0.0;
    std::vector<std::pair<double, std::vector<double>>> buffer;
    std::vector<double> average;
    // KALMAN
    int order = 0, n = 0, steps = 0;
    double time_step = 0.0, last_update = 0.0;
    std::vector<double> measurement;
    KalmanFilter filter;
    Mat prediction;   // [steps + 1][n] (column i of m_prediction as a row)

    void average_clear(double time)   // clear_old_measurements (forecast.cpp:67-86)
    {
        size_t it = 0;
        while (it < buffer.size() && !(time - window < buffer[it].first)) it++;
        buffer.erase(buffer.begin(), buffer.begin() + (long)it);
    }
    void average_update()   // update_average (forecast.cpp:88-101)
    {
        if (buffer.empty()) {
            std::fill(average.begin(), average.end(), 0.0);
            return;
        }
        std::vector<double> total = buffer[0].second;
        for (size_t i = 1; i < buffer.size(); i++)
            for (size_t k = 0; k < total.size(); k++) total[k] += buffer[i].second[k];
        for (size_t k = 0; k < total.size(); k++) average[k] = total[k] / (double)buffer.size();
    }
};

}   // namespace

extern "C" {

// Forecast::create; returns nullptr (and a message in *err) on the reference's failures.
void *oracle_forecast_create(const mppi_forecast_config *c, char *err, int errlen)
{
    auto fail = [&](const char *m) -> void * {
        if (err && errlen > 0) { std::strncpy(err, m, (size_t)errlen - 1); err[errlen - 1] = 0; }
        return nullptr;
    };
    OForecast *f = new OForecast();
    f->type = c->type;
    if (c->type == MPPI_FORECAST_LOCF) {
        f->observation.assign(c->locf_observation, c->locf_observation + 6);
        f->horison = c->locf_horison;
        f->valid_until = 0.0;
    } else if (c->type == MPPI_FORECAST_AVERAGE) {
        if (c->average_window < 0.0) { delete f; return fail("prediction window time is negative"); }
        f->window = c->average_window;
        f->average.assign((size_t)c->average_states, 0.0);
        f->last = 0.0;
    } else if (c->type == MPPI_FORECAST_KALMAN) {
        const int order = c->kalman_order, obs = c->kalman_observed_states;
        const int n = obs * (order + 1);
        f->order = order;
        f->n = n;
        f->time_step = c->kalman_time_step;
        f->horison = c->kalman_horison;
        f->steps = (int)std::ceil(c->kalman_horison / c->kalman_time_step);
        f->last_update = -c->kalman_time_step;
        f->measurement.assign((size_t)n, 0.0);
        KalmanFilter &k = f->filter;
        k.n = n;
        k.F.assign((size_t)n * n, 0.0);   // create_euler_state_transition_matrix (forecast.cpp:238-285)
        for (int d = 0; d <= order; d++)
            for (int s = 0; s < obs; s++) {
                const int row = d * obs + s;
                for (int i = 0; i <= order - d; i++) {
                    const int col = d * obs + i * obs + s;
                    k.F[(size_t)row * n + col] = 1.0 / (double)factorial((unsigned)i) * std::pow(c->kalman_time_step, (double)i);
                }
            }
        k.Q.assign((size_t)n * n, 0.0);
        k.R.assign((size_t)n * n, 0.0);
        k.P.assign((size_t)n * n, 0.0);
        for (int i = 0; i < n; i++) k.Q[(size_t)i * n + i] = k.R[(size_t)i * n + i] = k.P[(size_t)i * n + i] = 1e-8;
        k.x.assign((size_t)n, 0.0);
        for (int i = 0; i < obs; i++) k.x[i] = c->kalman_initial_state[i];
        k.xn = k.mul(k.F, k.x);   // KalmanFilter(config): m_next_state = F * initial_state
        f->prediction.assign((size_t)(f->steps + 1) * n, 0.0);
    } else {
        delete f;
        return fail("unknown forecast type");
    }
    return f;
}

void oracle_forecast_destroy(void *h) { delete (OForecast *)h; }

// Forecast::update(measurement, time)
void oracle_forecast_observe(void *h, const double *m, double time)
{
    OForecast *f = (OForecast *)h;
    if (f->type == MPPI_FORECAST_LOCF) {   // forecast.hpp:96-100
        f->valid_until = time + f->horison;
        f->observation.assign(m, m + 6);
    } else if (f->type == MPPI_FORECAST_AVERAGE) {   // forecast.cpp:109-122
        if (time < f->last) return;
        f->last = time;
        f->buffer.emplace_back(time, std::vector<double>(m, m + f->average.size()));
        f->average_clear(time);
        f->average_update();
    } else {   // KalmanForecast::update (forecast.cpp:298-331)
        const double dt = time - f->last_update;
        double delta[6];
        for (int k = 0; k < 6; k++) delta[k] = (m[k] - f->measurement[k]) / dt;
        for (int i = 1; i <= f->order; i++) {
            double next[6];
            for (int k = 0; k < 6; k++) next[k] = (delta[k] - f->measurement[(size_t)(6 * i + k)]) / dt;
            for (int k = 0; k < 6; k++) f->measurement[(size_t)(6 * i + k)] = delta[k];
            for (int k = 0; k < 6; k++) delta[k] = next[k];
        }
        for (int k = 0; k < 6; k++) f->measurement[k] = m[k];
        f->last_update = time;
        f->filter.update(f->measurement);
        KalmanFilter pred = f->filter;   // set_estimation / set_covariance
        pred.xn = pred.mul(pred.F, pred.x);
        const int n = f->n;
        for (int i = 0; i < n; i++) f->prediction[(size_t)i] = pred.x[i];
        for (int s = 0; s < f->steps; s++) {
            pred.predict(false);
            for (int i = 0; i < n; i++) f->prediction[(size_t)(s + 1) * n + i] = pred.x[i];
        }
    }
}

// Forecast::update(time)
void oracle_forecast_observe_time(void *h, double time)
{
    OForecast *f = (OForecast *)h;
    if (f->type == MPPI_FORECAST_AVERAGE) {   // forecast.cpp:102-107
        f->average_clear(time);
        f->average_update();
    } else if (f->type == MPPI_FORECAST_KALMAN) {   // forecast.cpp:333-340
        if (time <= f->last_update) return;
        f->filter.predict(true);
    }
}

// Forecast::forecast(time): the wrench (6)
void oracle_forecast_get(void *h, double time, double *out)
{
    OForecast *f = (OForecast *)h;
    if (f->type == MPPI_FORECAST_LOCF) {   // forecast.hpp:109-114
        for (int k = 0; k < 6; k++) out[k] = (time > f->valid_until) ? 0.0 : f->observation[(size_t)k];
    } else if (f->type == MPPI_FORECAST_AVERAGE) {
        for (int k = 0; k < 6; k++) out[k] = (size_t)k < f->average.size() ? f->average[(size_t)k] : 0.0;
    } else {   // forecast.cpp:342-367
        if (time > f->last_update + f->horison) {
            for (int k = 0; k < 6; k++) out[k] = 0.0;
            return;
        }
        double t = (time - f->last_update) / f->time_step;
        int lower = (int)t;
        t -= lower;
        lower = lower < 0 ? 0 : (lower > f->steps ? f->steps : lower);
        const int upper = lower + 1 > f->steps ? f->steps : lower + 1;
        const int n = f->n;
        for (int k = 0; k < 6; k++)
            out[k] = (1.0 - t) * f->prediction[(size_t)lower * n + k] + t * f->prediction[(size_t)upper * n + k];
    }
}

}   // extern "C"
