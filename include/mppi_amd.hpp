// mppi_amd.hpp — header-only C++ drop-in for the reference's src/controller/mppi.hpp, over the
// C-ABI of mppi_amd.h (link libmppi_amd.so).
//
// Same class names, member names, argument meaning and error behaviour as the reference:
//   mppi::Dynamics / Cost / Filter  mppi.hpp:30-176    the reference's pure virtuals, unchanged, so a
//                                                       plugin written against the reference compiles
//   mppi::DeviceDynamics / DeviceCost                   mixin: the device descriptor the kernels
//                                                       evaluate; create() refuses plugins without it
//                                                       (there is no CPU rollout path)
//   mppi::Configuration             mppi.hpp:181-249   (Eigen members -> std::vector, column-major)
//   mppi::Trajectory                mppi.hpp:267-658   (create returns nullptr + stderr on error;
//                                                       optimise()'s "all nan rollouts" throws)
//   FrankaRidgeback::PinocchioDynamics, AssistedManipulation, TrackPoint, DynamicsForecast: the
//   reference's plugins, their methods run on the device (mppi_dynamics_*, mppi_cost_evaluate).
// Vector types: Eigen's when <Eigen/Dense> is available (the reference's own signatures), else
// mppi::VectorXd / mppi::Ref below, which carry the data() / size() / operator[] the engine uses.
// Trajectory's update / get take anything with data() / size().
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <iostream>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "mppi_amd.h"
#include "mppi_amd_frankaridgeback.h"

#if __has_include(<Eigen/Dense>)
#include <Eigen/Dense>
namespace mppi {
using VectorXd = Eigen::VectorXd;
template <class T>
using Ref = Eigen::Ref<T>;
}  // namespace mppi
#else
namespace mppi {
// An owning dense vector of doubles (the part of Eigen::VectorXd the plugin surface needs).
class VectorXd {
public:
    VectorXd() = default;
    explicit VectorXd(std::ptrdiff_t n) : m_v((size_t)n, 0.0) {}
    VectorXd(std::initializer_list<double> l) : m_v(l) {}
    static VectorXd Zero(std::ptrdiff_t n) { return VectorXd(n); }
    double *data() { return m_v.data(); }
    const double *data() const { return m_v.data(); }
    std::ptrdiff_t size() const { return (std::ptrdiff_t)m_v.size(); }
    double &operator[](std::ptrdiff_t i) { return m_v[(size_t)i]; }
    double operator[](std::ptrdiff_t i) const { return m_v[(size_t)i]; }
    double &operator()(std::ptrdiff_t i) { return m_v[(size_t)i]; }
    double operator()(std::ptrdiff_t i) const { return m_v[(size_t)i]; }
    void resize(std::ptrdiff_t n) { m_v.assign((size_t)n, 0.0); }
    void setZero() { std::fill(m_v.begin(), m_v.end(), 0.0); }

private:
    std::vector<double> m_v;
};
// A non-owning view of a vector (Eigen::Ref<VectorXd>): what step() / get_state() return.
template <class T>
class Ref {
public:
    Ref(T &v) : m_p(v.data()), m_n(v.size()) {}
    Ref(double *p, std::ptrdiff_t n) : m_p(p), m_n(n) {}
    double *data() const { return m_p; }
    std::ptrdiff_t size() const { return m_n; }
    double &operator[](std::ptrdiff_t i) const { return m_p[i]; }
    double &operator()(std::ptrdiff_t i) const { return m_p[i]; }

private:
    double *m_p;
    std::ptrdiff_t m_n;
};
}  // namespace mppi
#endif

namespace mppi {

// mppi::Dynamics (mppi.hpp:30-85): the reference's pure virtuals.
class Dynamics {
public:
    virtual ~Dynamics() = default;
    virtual std::unique_ptr<Dynamics> copy() = 0;                             // :47
    virtual Ref<VectorXd> step(const VectorXd &control, double dt) = 0;      // :58
    virtual void set_state(const VectorXd &state, double time) = 0;          // :66
    virtual Ref<VectorXd> get_state() = 0;                                    // :72
    virtual int get_control_dof() = 0;                                        // :78
    virtual int get_state_dof() = 0;                                          // :84
};

// mppi::Cost (mppi.hpp:93-145).
class Cost {
public:
    virtual ~Cost() = default;
    virtual std::unique_ptr<Cost> copy() = 0;                                 // :110
    virtual void reset(double time) = 0;                                      // :115
    virtual double get_cost(const VectorXd &state, const VectorXd &control, Dynamics *dynamics,
                            double time) = 0;                                 // :127-132
    virtual int get_control_dof() = 0;                                        // :138
    virtual int get_state_dof() = 0;                                          // :144
};

// mppi::Filter (mppi.hpp:150-176).
class Filter {
public:
    virtual ~Filter() = default;
    virtual VectorXd filter(Ref<VectorXd> state, Ref<VectorXd> control, double time) = 0;   // :163-167
    virtual void reset(Ref<VectorXd> state, double time) = 0;                                // :175
};

// The device descriptors a plugin provides so the rollout kernels can evaluate it (the plugin's
// own step / get_cost are the host-callable methods; the rollouts never call back into the host).
class DeviceDynamics {
public:
    virtual ~DeviceDynamics() = default;
    virtual bool describe(mppi_dynamics_desc &out) const = 0;
};
class DeviceCost {
public:
    virtual ~DeviceCost() = default;
    virtual bool describe(mppi_cost_desc &out) const = 0;
    // the optimal rollout's per-term totals after an update (mppi_optimal_terms), for plugins that
    // keep the reference's accumulators (AssistedManipulation); the default ignores them
    virtual void set_optimal_terms(const double *) {}
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
        if (filter) {   // the reference's Actor passes nullptr (actor.cpp:100); the safety filter is stubs
            std::cerr << "mppi_amd: trajectory filters are not supported on the device" << std::endl;
            return nullptr;
        }
        mppi_dynamics_desc dd{};
        mppi_cost_desc cd{};
        const DeviceDynamics *ddev = dynamic_cast<const DeviceDynamics *>(dynamics.get());
        const DeviceCost *cdev = dynamic_cast<const DeviceCost *>(cost.get());
        if (!ddev || !ddev->describe(dd) || !cdev || !cdev->describe(cd)) {
            std::cerr << "mppi_amd: dynamics and cost must provide a device descriptor (mppi::DeviceDynamics / "
                         "mppi::DeviceCost); there is no CPU rollout path" << std::endl;
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

    // Thread 0's cost after filter() (mppi.hpp:448-454): BaseTest downcasts it to read the per-term
    // totals (base.cpp:140-146), so a cost that keeps them gets the optimal rollout's here.
    const Cost &get_optimal_cost() const
    {
        if (DeviceCost *dc = dynamic_cast<DeviceCost *>(m_cost.get())) {
            double t[7];
            if (mppi_optimal_terms(m_h, t) == MPPI_OK) dc->set_optimal_terms(t);
        }
        return *m_cost;
    }
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
    void forecast_table(double t0, double dt, int64_t steps, double *out) { check(mppi_forecast_table(m_h, t0, dt, steps, out)); }
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

// EndEffectorState (dynamics.hpp:95-117); orientation as (x, y, z, w) and as a row-major matrix.
struct EndEffectorState {
    double position[3];
    double orientation[4];
    double rotation[9];
    double linear_velocity[3], angular_velocity[3];
    double linear_acceleration[3], angular_acceleration[3];
    double jacobian[72];   // 6 x 12 row-major, WORLD

    static EndEffectorState from_row(const double *r)
    {
        EndEffectorState s{};
        std::copy(r + MPPI_EE_POSITION, r + MPPI_EE_POSITION + 3, s.position);
        std::copy(r + MPPI_EE_QUATERNION, r + MPPI_EE_QUATERNION + 4, s.orientation);
        std::copy(r + MPPI_EE_ROTATION, r + MPPI_EE_ROTATION + 9, s.rotation);
        std::copy(r + MPPI_EE_LINEAR_VELOCITY, r + MPPI_EE_LINEAR_VELOCITY + 3, s.linear_velocity);
        std::copy(r + MPPI_EE_ANGULAR_VELOCITY, r + MPPI_EE_ANGULAR_VELOCITY + 3, s.angular_velocity);
        std::copy(r + MPPI_EE_LINEAR_ACCELERATION, r + MPPI_EE_LINEAR_ACCELERATION + 3, s.linear_acceleration);
        std::copy(r + MPPI_EE_ANGULAR_ACCELERATION, r + MPPI_EE_ANGULAR_ACCELERATION + 3, s.angular_acceleration);
        std::copy(r + MPPI_EE_JACOBIAN, r + MPPI_EE_JACOBIAN + 72, s.jacobian);
        return s;
    }
};

// FrankaRidgeback::PinocchioDynamics (pinocchio_dynamics.hpp:30-427).  The rollouts evaluate the
// body table (describe(): generated from robot.urdf by default); the object itself, when its
// methods are called, is a device object (mppi_dynamics_*) created at the first call with the
// configuration's initial state (the constructor's set_state, pinocchio_dynamics.cpp:84-115).
class PinocchioDynamics : public mppi::Dynamics, public mppi::DeviceDynamics {
public:
    struct Configuration {
        std::vector<double> initial_state;   // State (31); HUDDLED when empty
        int device = 0;
    };
    // wrench forecast(time) of the dynamics' forecast handle (DynamicsForecast::Handle), or none
    using WrenchSource = std::function<bool(double time, double *wrench6)>;

    PinocchioDynamics() { mppi_frankaridgeback_model(&m_model); }
    explicit PinocchioDynamics(const mppi_frankaridgeback_desc &model) : m_model(model) {}
    PinocchioDynamics(const mppi_frankaridgeback_desc &model, const Configuration &c) : m_model(model), m_configuration(c) {}
    static std::unique_ptr<PinocchioDynamics> create(const Configuration &c)
    {
        mppi_frankaridgeback_desc m;
        mppi_frankaridgeback_model(&m);
        return std::make_unique<PinocchioDynamics>(m, c);
    }
    ~PinocchioDynamics() override { mppi_dynamics_destroy(m_obj); }

    std::unique_ptr<mppi::Dynamics> copy() override
    {
        auto d = std::make_unique<PinocchioDynamics>(m_model, m_configuration);
        d->m_forecast = m_forecast;
        return d;
    }
    mppi::Ref<mppi::VectorXd> step(const mppi::VectorXd &control, double dt) override
    {
        if (control.size() != MPPI_FR_CONTROL) throw std::invalid_argument("control has the wrong dimension");
        check(mppi_dynamics_step(object(), control.data(), dt, m_state.data()));
        return m_state;
    }
    void set_state(const mppi::VectorXd &state, double time) override
    {
        if (state.size() != MPPI_FR_STATE) throw std::invalid_argument("state has the wrong dimension");
        check(mppi_dynamics_set_state(object(), state.data(), time));
        check(mppi_dynamics_get_state(m_obj, m_state.data()));
    }
    mppi::Ref<mppi::VectorXd> get_state() override
    {
        check(mppi_dynamics_get_state(object(), m_state.data()));
        return m_state;
    }
    int get_control_dof() override { return MPPI_FR_CONTROL; }
    int get_state_dof() override { return MPPI_FR_STATE; }
    bool describe(mppi_dynamics_desc &out) const override
    {
        out = mppi_dynamics_desc{};
        out.kind = MPPI_DYNAMICS_FRANKARIDGEBACK;
        out.frankaridgeback = m_model;
        return true;
    }

    // FrankaRidgeback::Dynamics queries (dynamics.hpp:416-537)
    EndEffectorState get_end_effector_state()
    {
        double r[MPPI_EE_N];
        check(mppi_dynamics_end_effector(object(), r));
        return EndEffectorState::from_row(r);
    }
    std::vector<double> get_joint_position() { return query(0, 12); }
    std::vector<double> get_joint_velocity() { return query(12, 12); }
    std::vector<double> get_joint_acceleration() { return query(24, 12); }
    double get_tank_energy() { return query(48, 1)[0]; }
    double get_joint_power() const { return 0.0; }       // pinocchio_dynamics.hpp:211-214
    double get_external_power() const { return 0.0; }    // :220-223
    void add_end_effector_simulated_wrench(const double *) {}   // :276 (a no-op)
    void set_forecast(WrenchSource source) { m_forecast = std::move(source); }
    const WrenchSource &get_forecast() const { return m_forecast; }

    mppi_frankaridgeback_desc &model() { return m_model; }
    mppi_dynamics *object()
    {
        if (!m_obj) {
            std::vector<double> x0 = m_configuration.initial_state;
            if (x0.empty()) {
                x0.assign(MPPI_FR_STATE, 0.0);
                mppi_frankaridgeback_huddled(x0.data());
            }
            mppi_dynamics_desc d;
            describe(d);
            check(mppi_dynamics_create(&d, x0.data(), m_configuration.device, &m_obj));
        }
        return m_obj;
    }

private:
    std::vector<double> query(int off, int n)
    {
        double q[MPPI_DYNAMICS_QUERY_N];
        check(mppi_dynamics_query(object(), q));
        return std::vector<double>(q + off, q + off + n);
    }
    static void check(mppi_status st)
    {
        if (st != MPPI_OK) throw std::runtime_error(mppi_last_error(nullptr));
    }

    mppi_frankaridgeback_desc m_model;
    Configuration m_configuration;
    mppi_dynamics *m_obj = nullptr;
    mppi::VectorXd m_state = mppi::VectorXd(MPPI_FR_STATE);
    WrenchSource m_forecast;
};

// FrankaRidgeback::AssistedManipulation (objective/assisted_manipulation.hpp:16-398): Configuration
// is the POD mirror of AssistedManipulation::Configuration; DEFAULT_CONFIGURATION by default.
// get_cost against a PinocchioDynamics runs on the device (mppi_cost_evaluate) and accumulates the
// reference's per-term totals (m_joint_cost += ..., .cpp:74-319) that get_*_cost() return.
class AssistedManipulation : public mppi::Cost, public mppi::DeviceCost {
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
    void reset(double time) override   // :24-35
    {
        m_initial_time = time;
        for (double &t : m_terms) t = 0.0;
        m_cost = 0.0;
    }
    double get_cost(const mppi::VectorXd &state, const mppi::VectorXd &control, mppi::Dynamics *dynamics,
                    double time) override
    {
        auto *d = dynamic_cast<PinocchioDynamics *>(dynamics);
        if (!d) throw std::invalid_argument("AssistedManipulation::get_cost needs FrankaRidgeback::PinocchioDynamics");
        double wrench[6], out[8];
        const bool have = d->get_forecast() && d->get_forecast()(time, wrench);
        mppi_cost_desc cd;
        describe(cd);
        const mppi_status st = mppi_cost_evaluate(&cd, d->object(), state.data(), control.data(), have ? wrench : nullptr, out);
        if (st != MPPI_OK) throw std::runtime_error(mppi_last_error(nullptr));
        for (int i = 0; i < 7; i++) m_terms[i] += out[1 + i];
        m_cost += out[0];
        return out[0];
    }
    int get_control_dof() override { return MPPI_FR_CONTROL; }
    int get_state_dof() override { return MPPI_FR_STATE; }
    bool describe(mppi_cost_desc &out) const override
    {
        out = mppi_cost_desc{};
        out.kind = MPPI_COST_ASSISTED_MANIPULATION;
        out.assisted_manipulation = m_configuration;
        return true;
    }
    void set_optimal_terms(const double *t) override
    {
        for (int i = 0; i < 7; i++) m_terms[i] = t[i];
    }
    // assisted_manipulation.hpp:232-258
    double get_joint_limit_cost() const { return m_terms[MPPI_TERM_JOINT_LIMIT]; }
    double get_self_collision_cost() const { return m_terms[MPPI_TERM_SELF_COLLISION]; }
    double get_workspace_cost() const { return m_terms[MPPI_TERM_WORKSPACE]; }
    double get_energy_tank_cost() const { return m_terms[MPPI_TERM_ENERGY_TANK]; }
    double get_joint_velocity_cost() const { return m_terms[MPPI_TERM_JOINT_VELOCITY]; }
    double get_trajectory_cost() const { return m_terms[MPPI_TERM_TRAJECTORY]; }
    double get_manipulability_cost() const { return m_terms[MPPI_TERM_MANIPULABILITY]; }
    const Configuration &get_configuration() const { return m_configuration; }

private:
    Configuration m_configuration;
    double m_terms[7] = {0, 0, 0, 0, 0, 0, 0};
    double m_initial_time = 0.0, m_cost = 0.0;
};

// FrankaRidgeback::TrackPoint (frankaridgeback/objective/track_point.hpp:16-215): the same
// create / copy surface; DEFAULT_CONFIGURATION is track_point.hpp:72-107.
class TrackPoint : public mppi::Cost, public mppi::DeviceCost {
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
    void reset(double) override {}
    double get_cost(const mppi::VectorXd &state, const mppi::VectorXd &control, mppi::Dynamics *dynamics, double) override
    {
        auto *d = dynamic_cast<PinocchioDynamics *>(dynamics);
        if (!d) throw std::invalid_argument("TrackPoint::get_cost needs FrankaRidgeback::PinocchioDynamics");
        mppi_cost_desc cd;
        describe(cd);
        double out[8];
        const mppi_status st = mppi_cost_evaluate(&cd, d->object(), state.data(), control.data(), nullptr, out);
        if (st != MPPI_OK) throw std::runtime_error(mppi_last_error(nullptr));
        return out[0];
    }
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

// FrankaRidgeback::DynamicsForecast (dynamics.hpp:122-387, dynamics.cpp:57-138).  The wrench
// forecast it owns in the reference is the trajectory's device forecast here: create() attaches
// the configuration's Forecast::Configuration to `owner` (the trajectory whose rollouts read it,
// as the Actor shares one DynamicsForecast between both, actor.cpp:70-89).
class DynamicsForecast {
public:
    struct Configuration {
        double time_step;
        double horison;
        mppi_forecast_config end_effector_wrench_forecast;
    };

    static std::unique_ptr<DynamicsForecast> create(const Configuration &configuration,
                                                    std::unique_ptr<PinocchioDynamics> &&dynamics, mppi::Trajectory &owner)
    {
        const double s = std::ceil(configuration.horison / configuration.time_step);
        if (!(s > 0)) {
            std::cerr << "time horison is too small for time step" << std::endl;   // dynamics.cpp:70-74
            return nullptr;
        }
        if (mppi_forecast_attach(owner.handle(), &configuration.end_effector_wrench_forecast) != MPPI_OK) {
            std::cerr << "failed to create forecast for end effector wrench" << std::endl;   // :62-67
            return nullptr;
        }
        return std::unique_ptr<DynamicsForecast>(new DynamicsForecast(configuration, std::move(dynamics), owner, (unsigned)s));
    }

    void observe_wrench(const double *wrench6, double time) { m_owner.observe_wrench(wrench6, time); }
    void observe_time(double time) { m_owner.observe_time(time); }

    // dynamics.cpp:104-138: one device launch for the horison
    void forecast(const std::vector<double> &state, double time)
    {
        std::vector<double> wrench((size_t)m_steps * 6);
        m_owner.forecast_table(time, m_configuration.time_step, m_steps, wrench.data());
        m_rows.assign((size_t)m_steps * MPPI_DF_N, 0.0);
        const mppi_status st = mppi_dynamics_forecast(m_dynamics->object(), state.data(), time, m_configuration.time_step,
                                                      m_steps, wrench.data(), m_rows.data());
        if (st != MPPI_OK) throw std::runtime_error(mppi_last_error(nullptr));
        m_last_forecast = time;
    }
    double get_last_forecast_time() const { return m_last_forecast; }
    std::vector<double> get_joint_position(unsigned step) const { return row(step, MPPI_DF_JOINT_POSITION, 12); }
    EndEffectorState get_end_effector_state(double time) const
    {
        return EndEffectorState::from_row(m_rows.data() + (size_t)parameterise(time) * MPPI_DF_N + MPPI_DF_END_EFFECTOR);
    }
    std::vector<double> get_end_effector_wrench(double time)   // dynamics.hpp:275-278: the forecast itself
    {
        std::vector<double> w(6);
        m_owner.forecast(time, w.data());
        return w;
    }
    std::vector<double> get_wrench(unsigned step) const { return row(step, MPPI_DF_WRENCH, 6); }
    double get_energy(unsigned step) const { return m_rows[(size_t)step * MPPI_DF_N + MPPI_DF_ENERGY]; }
    double get_time_step() const { return m_configuration.time_step; }
    double get_horison() const { return m_configuration.horison; }
    unsigned get_steps() const { return m_steps; }
    // a wrench source for PinocchioDynamics::set_forecast (DynamicsForecast::Handle)
    PinocchioDynamics::WrenchSource handle()
    {
        return [this](double time, double *w) {
            m_owner.forecast(time, w);
            return true;
        };
    }

private:
    DynamicsForecast(const Configuration &c, std::unique_ptr<PinocchioDynamics> &&d, mppi::Trajectory &owner, unsigned steps)
        : m_configuration(c), m_dynamics(std::move(d)), m_owner(owner), m_steps(steps)
    {
    }
    std::int64_t parameterise(double time) const   // dynamics.hpp:344-359, literally
    {
        if (time < m_last_forecast) return 0;
        if (time >= m_configuration.horison) return m_steps - 1;
        return (std::int64_t)((time - m_last_forecast) / m_configuration.time_step);
    }
    std::vector<double> row(unsigned step, int off, int n) const
    {
        const double *r = m_rows.data() + (size_t)step * MPPI_DF_N + off;
        return std::vector<double>(r, r + n);
    }

    Configuration m_configuration;
    std::unique_ptr<PinocchioDynamics> m_dynamics;
    mppi::Trajectory &m_owner;
    unsigned m_steps;
    double m_last_forecast = 2.2250738585072014e-308;   // std::numeric_limits<double>::min()
    std::vector<double> m_rows;
};

}  // namespace FrankaRidgeback
