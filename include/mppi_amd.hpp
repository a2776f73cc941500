// mppi_amd.hpp — header-only C++ drop-in for the reference's src/controller/mppi.hpp, over the
// C-ABI of mppi_amd.h (link libmppi_amd.so).
//
// Same class names, member names, argument meaning and error behaviour as the reference:
//   mppi::Configuration          mppi.hpp:181-249   (Eigen members -> std::vector, column-major)
//   mppi::Dynamics / mppi::Cost  mppi.hpp:30-145    (+ describe(): the device descriptor)
//   mppi::Filter                 mppi.hpp:150-176   (accepted only as nullptr, as the Actor does)
//   mppi::Trajectory             mppi.hpp:267-658   (create returns nullptr + stderr on error;
//                                                   optimise()'s "all nan rollouts" throws)
//   FrankaRidgeback::PinocchioDynamics / FrankaRidgeback::AssistedManipulation plugins.
// Vector arguments are templates over anything with data()/size() — Eigen::VectorXd,
// Eigen::Ref<VectorXd>, std::vector<double> — so the reference's call sites compile unchanged.
// Plugins without a device descriptor are rejected at create(): there is no CPU fallback.
#pragma once

#include <cstdint>
#include <cstdio>
#include <iostream>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "mppi_amd.h"
#include "mppi_amd_frankaridgeback.h"

namespace mppi {

class Dynamics {
public:
    virtual ~Dynamics() = default;
    virtual std::unique_ptr<Dynamics> copy() = 0;
    virtual int get_control_dof() = 0;
    virtual int get_state_dof() = 0;
    // Device descriptor evaluated by the rollout kernels; false = not device-describable.
    virtual bool describe(mppi_dynamics_desc &out) const = 0;
};

class Cost {
public:
    virtual ~Cost() = default;
    virtual std::unique_ptr<Cost> copy() = 0;
    virtual void reset(double) {}
    virtual int get_control_dof() = 0;
    virtual int get_state_dof() = 0;
    virtual bool describe(mppi_cost_desc &out) const = 0;
};

class Filter {
public:
    virtual ~Filter() = default;
};

struct Configuration {
    std::vector<double> initial_state;
    std::int64_t rollouts = 0;
    std::int64_t keep_best_rollouts = 0;
    double time_step = 0.01;
    double horison = 0.0;
    double gradient_step = 1.0;
    double cost_scale = 1.0;
    double cost_discount_factor = 1.0;
    std::vector<double> covariance;   // C x C, column-major (Eigen's default)
    bool control_bound = false;
    std::vector<double> control_min;
    std::vector<double> control_max;
    std::optional<std::vector<double>> control_default;
    struct Smoothing {
        unsigned int window;
        unsigned int order;
    };
    std::optional<Smoothing> smoothing;
    unsigned int threads = 1;
};

class Trajectory {
public:
    struct Rollout {
        std::vector<double> noise;   // C x H column-major
        double cost;
    };

    static std::unique_ptr<Trajectory> create(const Configuration &configuration, std::unique_ptr<Dynamics> &&dynamics,
                                              std::unique_ptr<Cost> &&cost, std::unique_ptr<Filter> &&filter = nullptr,
                                              int device = 0)
    {
        if (filter) {
            std::cerr << "mppi_amd: trajectory filters are not supported on the device" << std::endl;
            return nullptr;
        }
        mppi_dynamics_desc dd{};
        mppi_cost_desc cd{};
        if (!dynamics || !dynamics->describe(dd) || !cost || !cost->describe(cd)) {
            std::cerr << "mppi_amd: dynamics and cost must provide a device descriptor" << std::endl;
            return nullptr;
        }
        mppi_config c{};
        c.initial_state = configuration.initial_state.data();
        c.state_dof = (int64_t)configuration.initial_state.size();
        c.control_dof = (int64_t)configuration.control_min.size();
        c.rollouts = configuration.rollouts;
        c.keep_best_rollouts = configuration.keep_best_rollouts;
        c.time_step = configuration.time_step;
        c.horison = configuration.horison;
        c.gradient_step = configuration.gradient_step;
        c.cost_scale = configuration.cost_scale;
        c.cost_discount_factor = configuration.cost_discount_factor;
        if (configuration.covariance.size() != (size_t)(c.control_dof * c.control_dof)) {
            std::cerr << "controller covariance matrix not square" << std::endl;
            return nullptr;
        }
        c.covariance = configuration.covariance.data();
        c.control_bound = configuration.control_bound;
        c.control_min = configuration.control_min.data();
        c.control_max = configuration.control_max.data();
        c.has_control_default = configuration.control_default.has_value();
        c.control_default = configuration.control_default ? configuration.control_default->data() : nullptr;
        c.has_smoothing = configuration.smoothing.has_value();
        c.smoothing_window = configuration.smoothing ? configuration.smoothing->window : 0;
        c.smoothing_order = configuration.smoothing ? configuration.smoothing->order : 0;
        c.threads = configuration.threads;
        mppi_handle *h = nullptr;
        if (mppi_create(&c, &dd, &cd, device, &h) != MPPI_OK) {
            std::cerr << mppi_last_error(nullptr) << std::endl;   // the reference prints and returns nullptr
            return nullptr;
        }
        return std::unique_ptr<Trajectory>(new Trajectory(h, configuration, std::move(dynamics), std::move(cost)));
    }

    ~Trajectory() { mppi_destroy(m_h); }
    Trajectory(const Trajectory &) = delete;
    Trajectory &operator=(const Trajectory &) = delete;

    // Trajectory::update (mppi.cpp:154-187).  Throws std::runtime_error("all nan rollouts") like
    // optimise(), and std::runtime_error for device / smoothing failures.
    template <class Vec>
    void update(const Vec &state, double time)
    {
        update_raw(state.data(), (size_t)state.size(), time);
    }

    void update_raw(const double *state, size_t n, double time)
    {
        if (n != (size_t)m_X) throw std::invalid_argument("state has the wrong dimension");
        check(mppi_update(m_h, state, time));
        m_rolled_out_state.assign(state, state + n);
        m_update_last = time;
        ++m_update_count;
    }

    // Trajectory::get (mppi.cpp:481-512): `control` is pre-sized (Eigen::Ref<VectorXd> in the
    // reference).
    template <class Vec>
    void get(Vec &&control, double time)
    {
        check(mppi_get(m_h, time, control.data()));
    }

    std::vector<double> operator()(double time)
    {
        std::vector<double> u((size_t)m_C);
        check(mppi_get(m_h, time, u.data()));
        return u;
    }

    unsigned int get_state_dof() const { return (unsigned int)m_X; }
    unsigned int get_control_dof() const { return (unsigned int)m_C; }
    double get_time_step() const { return m_configuration.time_step; }
    unsigned int get_step_count() const { return (unsigned int)m_H; }
    double get_update_duration() const
    {
        double d = 0;
        mppi_update_duration(m_h, &d);
        return d;
    }
    double get_update_last() const { return m_update_last; }
    std::size_t get_update_count() const { return m_update_count; }
    std::size_t get_rollout_count() const { return (std::size_t)m_R; }
    const std::vector<double> &get_rolled_out_state() const { return m_rolled_out_state; }

    std::vector<double> get_weights() const { return fetch(mppi_weights, (size_t)m_R); }
    std::vector<double> get_gradient() const { return fetch(mppi_gradient, (size_t)(m_C * m_H)); }
    std::vector<double> get_optimal_rollout() const { return fetch(mppi_optimal_control, (size_t)(m_C * m_H)); }
    std::vector<double> trajectory() const { return get_optimal_rollout(); }
    std::vector<double> get_costs() const { return fetch(mppi_costs, (size_t)m_R); }

    std::vector<Rollout> get_rollouts() const
    {
        std::vector<double> n = fetch(mppi_noise, (size_t)(m_R * m_C * m_H));
        std::vector<double> c = get_costs();
        std::vector<Rollout> out((size_t)m_R);
        for (int64_t r = 0; r < m_R; r++) {
            out[(size_t)r].noise.assign(n.begin() + r * m_C * m_H, n.begin() + (r + 1) * m_C * m_H);
            out[(size_t)r].cost = c[(size_t)r];
        }
        return out;
    }

    double get_optimal_total_cost() const
    {
        double c = 0;
        mppi_optimal_cost(m_h, &c);
        return c;
    }

    const Cost &get_optimal_cost() const { return *m_cost; }
    const Dynamics &get_optimal_dynamics() const { return *m_dynamics; }

    // Per-update inputs and parity hooks of the device engine.
    template <class Vec>
    void set_forecast(const Vec &wrench_Hx6) { check(mppi_set_forecast(m_h, wrench_Hx6.data())); }
    void set_noise_source(int source, uint64_t seed = 0x5EED) { check(mppi_set_noise_source(m_h, source, seed)); }
    // The wrench forecast on the device (DynamicsForecast::observe_wrench / observe_time and
    // Forecast::forecast, dynamics.hpp:221-278): every update samples it at t0 + k dt.
    void attach_forecast(const mppi_forecast_config *configuration) { check(mppi_forecast_attach(m_h, configuration)); }
    void observe_wrench(const double *wrench6, double time) { check(mppi_forecast_observe(m_h, wrench6, time)); }
    void observe_time(double time) { check(mppi_forecast_observe_time(m_h, time)); }
    void forecast(double time, double *wrench6) { check(mppi_forecast_get(m_h, time, wrench6)); }
    mppi_handle *handle() const { return m_h; }

private:
    Trajectory(mppi_handle *h, const Configuration &c, std::unique_ptr<Dynamics> &&d, std::unique_ptr<Cost> &&k)
        : m_h(h), m_configuration(c), m_dynamics(std::move(d)), m_cost(std::move(k))
    {
        mppi_dims(m_h, &m_R, &m_H, &m_C, &m_X);
        m_rolled_out_state.assign((size_t)m_X, 0.0);   // m_rollout_state.setZero() (mppi.cpp:121)
    }

    void check(mppi_status st) const
    {
        if (st == MPPI_OK) return;
        throw std::runtime_error(st == MPPI_ERR_ALL_NAN ? std::string("all nan rollouts") : std::string(mppi_last_error(m_h)));
    }

    template <class F>
    std::vector<double> fetch(F fn, size_t n) const
    {
        std::vector<double> v(n);
        check(fn(m_h, v.data()));
        return v;
    }

    mppi_handle *m_h;
    Configuration m_configuration;
    std::unique_ptr<Dynamics> m_dynamics;
    std::unique_ptr<Cost> m_cost;
    int64_t m_R = 0, m_H = 0, m_C = 0, m_X = 0;
    std::vector<double> m_rolled_out_state;
    double m_update_last = 0;
    std::size_t m_update_count = 0;
};

}  // namespace mppi

namespace FrankaRidgeback {

// FrankaRidgeback::PinocchioDynamics (pinocchio_dynamics.hpp:30): the body table generated from
// robot.urdf (mppi_amd_frankaridgeback.h) by default.
class PinocchioDynamics : public mppi::Dynamics {
public:
    PinocchioDynamics() { mppi_frankaridgeback_model(&m_model); }
    explicit PinocchioDynamics(const mppi_frankaridgeback_desc &model) : m_model(model) {}
    std::unique_ptr<mppi::Dynamics> copy() override { return std::make_unique<PinocchioDynamics>(m_model); }
    int get_control_dof() override { return MPPI_FR_CONTROL; }
    int get_state_dof() override { return MPPI_FR_STATE; }
    bool describe(mppi_dynamics_desc &out) const override
    {
        out = mppi_dynamics_desc{};
        out.kind = MPPI_DYNAMICS_FRANKARIDGEBACK;
        out.frankaridgeback = m_model;
        return true;
    }
    mppi_frankaridgeback_desc &model() { return m_model; }

private:
    mppi_frankaridgeback_desc m_model;
};

// FrankaRidgeback::AssistedManipulation (objective/assisted_manipulation.hpp:16): Configuration is
// the POD mirror of AssistedManipulation::Configuration; DEFAULT_CONFIGURATION by default.
class AssistedManipulation : public mppi::Cost {
public:
    using Configuration = mppi_assisted_manipulation_desc;
    static Configuration default_configuration()
    {
        Configuration c;
        mppi_assisted_manipulation_default(&c);
        return c;
    }
    static std::unique_ptr<AssistedManipulation> create(const Configuration &c)
    {
        return std::make_unique<AssistedManipulation>(c);
    }
    AssistedManipulation() : m_configuration(default_configuration()) {}
    explicit AssistedManipulation(const Configuration &c) : m_configuration(c) {}
    std::unique_ptr<mppi::Cost> copy() override { return std::make_unique<AssistedManipulation>(m_configuration); }
    int get_control_dof() override { return MPPI_FR_CONTROL; }
    int get_state_dof() override { return MPPI_FR_STATE; }
    bool describe(mppi_cost_desc &out) const override
    {
        out = mppi_cost_desc{};
        out.kind = MPPI_COST_ASSISTED_MANIPULATION;
        out.assisted_manipulation = m_configuration;
        return true;
    }

private:
    Configuration m_configuration;
};

// FrankaRidgeback::TrackPoint (frankaridgeback/objective/track_point.hpp:16-215): the same
// create / copy surface; DEFAULT_CONFIGURATION is track_point.hpp:72-107.
class TrackPoint : public mppi::Cost {
public:
    using Configuration = mppi_track_point_desc;
    static Configuration default_configuration()
    {
        Configuration c;
        mppi_track_point_default(&c);
        return c;
    }
    static inline const Configuration DEFAULT_CONFIGURATION = default_configuration();
    static std::unique_ptr<TrackPoint> create(const Configuration &c) { return std::make_unique<TrackPoint>(c); }
    TrackPoint() : m_configuration(default_configuration()) {}
    explicit TrackPoint(const Configuration &c) : m_configuration(c) {}
    std::unique_ptr<mppi::Cost> copy() override { return std::make_unique<TrackPoint>(m_configuration); }
    int get_control_dof() override { return MPPI_FR_CONTROL; }
    int get_state_dof() override { return MPPI_FR_STATE; }
    bool describe(mppi_cost_desc &out) const override
    {
        out = mppi_cost_desc{};
        out.kind = MPPI_COST_TRACK_POINT;
        out.track_point = m_configuration;
        return true;
    }

private:
    Configuration m_configuration;
};

}  // namespace FrankaRidgeback
