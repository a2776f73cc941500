// sanitize_check.cpp — TEST INFRASTRUCTURE: drives the CPU oracle's C API through every path the
// tests use, built with -fsanitize=address,undefined -fno-sanitize-recover=all (oracle/Makefile
// `sanitize`, SURVEY §5 "Race detection / sanitizers"; the reference itself builds with -Wall only,
// src/CMakeLists.txt:8).  Any out-of-bounds access, use-after-free, leak or undefined behaviour
// aborts with a report; the checks below only guard that each path ran and produced numbers.
//
// Paths: config-1 updates with uint8 index semantics (mppi.cpp quirks), wide indices with NaN
// rollouts, Savitzky-Golay smoothing, the energy tank, TrackPoint, the sharded mode's all-reduce
// callback, two threads, the Pinocchio-order vs minimal-arithmetic dynamics, the forecast oracle
// (LOCF / Average / Kalman), the PinocchioDynamics object and get_cost against it, the FLOP counter.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../include/mppi_amd.h"
#include "../include/mppi_amd_frankaridgeback.h"

extern "C" {
void *oracle_create(const mppi_config *, const mppi_dynamics_desc *, const mppi_cost_desc *, int, int, int);
void oracle_destroy(void *);
const char *oracle_last_error(void *);
void oracle_set_noise_source(void *, int, uint64_t);
void oracle_inject_noise(void *, const double *, int64_t);
int64_t oracle_noise_draws(void *, double);
void oracle_set_forecast(void *, const double *);
int oracle_update(void *, const double *, double);
void oracle_costs(void *, double *);
void oracle_weights(void *, double *);
void oracle_gradient(void *, double *);
void oracle_optimal_control(void *, double *);
void oracle_noise(void *, double *);
void oracle_optimal_terms(void *, double *);
double oracle_optimal_cost(void *);
void oracle_set_threads(void *, unsigned);
void oracle_set_shard(void *, int64_t, int64_t, void (*)(double *, int64_t));
void oracle_dims(void *, int64_t *, int64_t *, int64_t *, int64_t *);
void oracle_smoothing_windows(void *, double *, double *, int64_t *);
int oracle_get(void *, double, double *);
void oracle_default_frankaridgeback(mppi_frankaridgeback_desc *);
void oracle_default_assisted_manipulation(mppi_assisted_manipulation_desc *);
double oracle_count_flops(const mppi_frankaridgeback_desc *, const mppi_assisted_manipulation_desc *, const double *, int64_t);
void *oracle_forecast_create(const mppi_forecast_config *, char *, int);
void oracle_forecast_destroy(void *);
void oracle_forecast_observe(void *, const double *, double);
void oracle_forecast_observe_time(void *, double);
void oracle_forecast_get(void *, double, double *);
void *oracle_dyn_create(const mppi_frankaridgeback_desc *, const double *);
void oracle_dyn_destroy(void *);
void oracle_dyn_step(void *, const double *, double, double *);
void oracle_dyn_end_effector(void *, double *);
void oracle_dyn_forecast(void *, const double *, double, double, int64_t, const double *, double *);
void oracle_cost_evaluate(const mppi_cost_desc *, void *, const double *, const double *, double *);
}

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) { std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); g_fail = 1; } \
    } while (0)

struct Setup {
    std::vector<double> x0, cov, cmin, cmax, cdef;
    mppi_config cfg{};
    mppi_dynamics_desc dyn{};
    mppi_cost_desc cost{};
    Setup(int64_t S, double horison, int64_t K, int smoothing = 0)
    {
        x0.assign(MPPI_FR_STATE, 0.0);
        mppi_frankaridgeback_huddled(x0.data());
        cov.assign(144, 0.0);
        for (int i = 0; i < 12; i++) cov[13 * i] = MPPI_FR_DEFAULT_VARIANCE[i];
        cmin.assign(MPPI_FR_DEFAULT_CONTROL_MIN, MPPI_FR_DEFAULT_CONTROL_MIN + 12);
        cmax.assign(MPPI_FR_DEFAULT_CONTROL_MAX, MPPI_FR_DEFAULT_CONTROL_MAX + 12);
        cdef.assign(12, 0.0);
        cfg.initial_state = x0.data();
        cfg.state_dof = MPPI_FR_STATE;
        cfg.control_dof = 12;
        cfg.rollouts = S;
        cfg.keep_best_rollouts = K;
        cfg.time_step = 0.01;
        cfg.horison = horison;
        cfg.gradient_step = 2.0;
        cfg.cost_scale = 10.0;
        cfg.cost_discount_factor = 1.0;
        cfg.covariance = cov.data();
        cfg.control_bound = 1;
        cfg.control_min = cmin.data();
        cfg.control_max = cmax.data();
        cfg.has_control_default = 1;
        cfg.control_default = cdef.data();
        cfg.has_smoothing = smoothing > 0;
        cfg.smoothing_window = (uint32_t)smoothing;
        cfg.smoothing_order = 1;
        cfg.threads = 2;
        dyn.kind = MPPI_DYNAMICS_FRANKARIDGEBACK;
        oracle_default_frankaridgeback(&dyn.frankaridgeback);
        cost.kind = MPPI_COST_ASSISTED_MANIPULATION;
        oracle_default_assisted_manipulation(&cost.assisted_manipulation);
    }
};

// injected-noise updates; returns the last costs
static std::vector<double> run(Setup &s, int mode, int compat, int updates, uint64_t seed, bool nan_noise = false)
{
    void *h = oracle_create(&s.cfg, &s.dyn, &s.cost, 0, mode, compat);
    CHECK(h != nullptr);
    if (!h) return {};
    int64_t R, H, C, X;
    oracle_dims(h, &R, &H, &C, &X);
    std::vector<double> table((size_t)(6 * H), 0.0);
    for (int64_t k = 0; k < H; k++) table[(size_t)(6 * k)] = 20.0;
    oracle_set_forecast(h, table.data());
    oracle_set_noise_source(h, 1, 0);
    std::mt19937_64 gen(seed);
    std::normal_distribution<double> nd(0.0, 1.0);
    for (int j = 0; j < updates; j++) {
        const double t = 0.05 * j;
        const int64_t n = oracle_noise_draws(h, t);
        std::vector<double> eps((size_t)(n * C));
        for (int64_t i = 0; i < n; i++)
            for (int64_t c = 0; c < C; c++) eps[(size_t)(i * C + c)] = nd(gen) * std::sqrt(MPPI_FR_DEFAULT_VARIANCE[c]);
        if (nan_noise && j == 1 && n > 40) eps[(size_t)(16 * C + 4)] = 1e300;   // a NaN rollout
        oracle_inject_noise(h, eps.data(), n);
        const int st = oracle_update(h, s.x0.data(), t);
        CHECK(st == 0);
        double u[12];
        CHECK(oracle_get(h, t + 0.013, u) == 0);
    }
    std::vector<double> costs((size_t)R), w((size_t)R), g((size_t)(H * C)), U((size_t)(H * C)), terms(7);
    std::vector<double> noise((size_t)(R * H * C));
    oracle_costs(h, costs.data());
    oracle_weights(h, w.data());
    oracle_gradient(h, g.data());
    oracle_optimal_control(h, U.data());
    oracle_noise(h, noise.data());
    oracle_optimal_terms(h, terms.data());
    CHECK(std::isfinite(oracle_optimal_cost(h)));
    for (double v : U) CHECK(std::isfinite(v));
    if (s.cfg.has_smoothing) {
        const int64_t W = H + 2 * s.cfg.smoothing_window + 1;
        std::vector<double> uu((size_t)(C * W)), tt((size_t)(C * W));
        std::vector<int64_t> st((size_t)C);
        oracle_smoothing_windows(h, uu.data(), tt.data(), st.data());
    }
    oracle_destroy(h);
    return costs;
}

static std::vector<double> *g_shard_sum = nullptr;
static void fake_allreduce(double *, int64_t) {}   // one rank: the sum is itself

int main()
{
    {   // config 1 with the reference's uint8 index semantics, two dynamics orders agree
        Setup s(128, 0.32, 20);
        std::vector<double> a = run(s, 0, 1, 3, 12345), b = run(s, 1, 1, 3, 12345);
        CHECK(a.size() == b.size());
        double mn = INFINITY, mx = -INFINITY, err = 0.0;
        for (size_t i = 0; i < a.size(); i++) {
            if (std::isnan(a[i])) continue;
            mn = std::fmin(mn, a[i]);
            mx = std::fmax(mx, a[i]);
            err = std::fmax(err, std::fabs(a[i] - b[i]));
        }
        CHECK(err <= 1e-11 * (mx - mn) + 1e-2);
    }
    {   // wide indices past 255 rollouts, NaN rollouts
        Setup s(300, 0.16, 8);
        std::vector<double> c = run(s, 0, 0, 3, 7, true);
        CHECK(!c.empty());
    }
    {   // Savitzky-Golay window 10 order 1
        Setup s(64, 0.32, 8, 10);
        run(s, 0, 0, 4, 3);
    }
    {   // energy tank, TrackPoint
        Setup s(64, 0.16, 8);
        s.cost.assisted_manipulation.enable_energy_limit = 1;
        s.x0[30] = 15.0;
        run(s, 0, 0, 3, 5);
        Setup t(64, 0.16, 8);
        t.cost.kind = MPPI_COST_TRACK_POINT;
        t.cost.track_point.point[0] = 0.8;
        t.cost.track_point.enable_joint_limits = t.cost.track_point.enable_reach_limits = 1;
        run(t, 0, 0, 3, 6);
    }
    {   // sharded mode (one rank: the whole range, the all-reduce callback a no-op)
        Setup s(64, 0.16, 8);
        void *h = oracle_create(&s.cfg, &s.dyn, &s.cost, 0, 0, 0);
        CHECK(h != nullptr);
        oracle_set_threads(h, 3);
        oracle_set_shard(h, 0, 66, fake_allreduce);
        oracle_set_noise_source(h, 1, 0);
        const int64_t n = oracle_noise_draws(h, 0.0);
        std::vector<double> eps((size_t)(n * 12), 0.1);
        oracle_inject_noise(h, eps.data(), n);
        CHECK(oracle_update(h, s.x0.data(), 0.0) == 0);
        oracle_destroy(h);
        (void)g_shard_sum;
    }
    {   // the forecast oracle: LOCF, Average, Kalman (order 2)
        char err[256];
        mppi_forecast_config c{};
        const double w[6] = {1, 2, 3, 0, 0, 0};
        double out[6];
        for (int type = 0; type < 3; type++) {
            std::memset(&c, 0, sizeof(c));
            c.type = type;
            c.locf_horison = 0.5;
            c.average_states = 6;
            c.average_window = 0.2;
            c.kalman_observed_states = 6;
            c.kalman_time_step = 0.01;
            c.kalman_horison = 0.3;
            c.kalman_order = 2;
            void *f = oracle_forecast_create(&c, err, sizeof(err));
            CHECK(f != nullptr);
            if (!f) continue;
            for (int i = 0; i < 20; i++) {
                oracle_forecast_observe(f, w, 0.01 * i);
                oracle_forecast_observe_time(f, 0.01 * i + 0.005);
            }
            oracle_forecast_get(f, 0.25, out);
            for (double v : out) CHECK(std::isfinite(v));
            oracle_forecast_destroy(f);
        }
    }
    {   // the PinocchioDynamics object, DynamicsForecast, get_cost against it, FLOP counter
        Setup s(16, 0.08, 4);
        void *d = oracle_dyn_create(&s.dyn.frankaridgeback, s.x0.data());
        double u[12] = {0.1, -0.1, 0.2, 5, -5, 3, -3, 1, -1, 2, 0, 0}, x[MPPI_FR_STATE], ee[MPPI_EE_N], c8[8];
        for (int k = 0; k < 10; k++) oracle_dyn_step(d, u, 0.01, x);
        oracle_dyn_end_effector(d, ee);
        for (double v : ee) CHECK(std::isfinite(v));
        std::vector<double> rows((size_t)(32 * MPPI_DF_N)), wr(32 * 6, 1.0);
        oracle_dyn_forecast(d, s.x0.data(), 0.1, 0.01, 32, wr.data(), rows.data());
        for (double v : rows) CHECK(std::isfinite(v));
        oracle_cost_evaluate(&s.cost, d, x, wr.data(), c8);
        CHECK(std::isfinite(c8[0]) && c8[0] > 0.0);
        oracle_dyn_destroy(d);
        CHECK(oracle_count_flops(&s.dyn.frankaridgeback, &s.cost.assisted_manipulation, s.x0.data(), 8) > 0.0);
    }
    std::printf("%s\n", g_fail ? "sanitize_check: FAILED" : "sanitize_check: ok");
    return g_fail;
}
