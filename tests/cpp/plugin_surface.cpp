// The reference's plugin surface through the C++ drop-in (include/mppi_amd.hpp):
//  - plugins written the reference's way (override of mppi.hpp:47-84, 110-144, 163-175) compile
//    against the shim; create() refuses those without a device descriptor, and any filter;
//  - with "gpu": FrankaRidgeback::PinocchioDynamics used through mppi::Dynamics* (set_state / step /
//    get_state on the device object), AssistedManipulation::get_cost against it, the optimal
//    rollout's per-term totals through get_optimal_cost()'s downcast (base.cpp:140-146), and
//    DynamicsForecast::forecast; printed as JSON lines for tests/test_cpp_dropin.py.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "mppi_amd.hpp"

namespace {

// A plugin written against the reference's interface (a double integrator, as in the README's
// "Subclass to implement dynamics"): no device descriptor.
class DoubleIntegrator : public mppi::Dynamics {
public:
    DoubleIntegrator() : m_state(6) {}
    std::unique_ptr<mppi::Dynamics> copy() override { return std::make_unique<DoubleIntegrator>(*this); }
    mppi::Ref<mppi::VectorXd> step(const mppi::VectorXd &control, double dt) override
    {
        for (int i = 0; i < 3; i++) {
            m_state[3 + i] += control[i] * dt;
            m_state[i] += m_state[3 + i] * dt;
        }
        return m_state;
    }
    void set_state(const mppi::VectorXd &state, double) override
    {
        for (int i = 0; i < 6; i++) m_state[i] = state[i];
    }
    mppi::Ref<mppi::VectorXd> get_state() override { return m_state; }
    int get_control_dof() override { return 3; }
    int get_state_dof() override { return 6; }

private:
    mppi::VectorXd m_state;
};

class Quadratic : public mppi::Cost {
public:
    std::unique_ptr<mppi::Cost> copy() override { return std::make_unique<Quadratic>(); }
    void reset(double) override {}
    double get_cost(const mppi::VectorXd &state, const mppi::VectorXd &, mppi::Dynamics *, double) override
    {
        double c = 0;
        for (int i = 0; i < 3; i++) c += state[i] * state[i];
        return c;
    }
    int get_control_dof() override { return 3; }
    int get_state_dof() override { return 6; }
};

class PassThrough : public mppi::Filter {
public:
    mppi::VectorXd filter(mppi::Ref<mppi::VectorXd>, mppi::Ref<mppi::VectorXd> control, double) override
    {
        mppi::VectorXd out(control.size());
        for (std::ptrdiff_t i = 0; i < control.size(); i++) out[i] = control[i];
        return out;
    }
    void reset(mppi::Ref<mppi::VectorXd>, double) override {}
};

mppi::Configuration fr_configuration(long rollouts, double horison)
{
    mppi::Configuration c;   // BaseTest::DEFAULT_CONFIGURATION's mppi block (base.hpp:69-101)
    c.initial_state.assign(MPPI_FR_STATE, 0.0);
    mppi_frankaridgeback_huddled(c.initial_state.data());
    c.rollouts = rollouts;
    c.keep_best_rollouts = 20;
    c.time_step = 0.01;
    c.horison = horison;
    c.gradient_step = 2.0;
    c.cost_scale = 10.0;
    c.cost_discount_factor = 1.0;
    c.covariance.assign(144, 0.0);
    for (int i = 0; i < 12; i++) c.covariance[13 * i] = MPPI_FR_DEFAULT_VARIANCE[i];
    c.control_bound = true;
    c.control_min.assign(MPPI_FR_DEFAULT_CONTROL_MIN, MPPI_FR_DEFAULT_CONTROL_MIN + 12);
    c.control_max.assign(MPPI_FR_DEFAULT_CONTROL_MAX, MPPI_FR_DEFAULT_CONTROL_MAX + 12);
    c.control_default = std::vector<double>(12, 0.0);
    c.threads = 36;
    return c;
}

void print_vec(const char *key, const double *v, int n, bool last = false)
{
    std::printf("\"%s\": [", key);
    for (int i = 0; i < n; i++) std::printf("%s%.17g", i ? ", " : "", v[i]);
    std::printf("]%s", last ? "" : ", ");
}

}  // namespace

int main(int argc, char **argv)
{
    const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
    {   // reference-shaped plugins: no device descriptor -> nullptr (no CPU rollout path)
        mppi::Configuration c;
        c.initial_state.assign(6, 0.0);
        c.rollouts = 16;
        c.time_step = 0.01;
        c.horison = 0.1;
        c.covariance = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        c.control_min = {-1, -1, -1};
        c.control_max = {1, 1, 1};
        std::unique_ptr<mppi::Dynamics> dyn = std::make_unique<DoubleIntegrator>();
        mppi::VectorXd x(6), u(3);
        x[0] = 1.0;
        u[0] = 2.0;
        dyn->set_state(x, 0.0);
        const double x0_after = dyn->step(u, 0.5)[0];   // 1 + (2 * 0.5) * 0.5
        if (std::fabs(x0_after - 1.5) > 1e-15) return 10;
        auto t = mppi::Trajectory::create(c, std::move(dyn), std::make_unique<Quadratic>());
        if (t) return 11;
        auto t2 = mppi::Trajectory::create(fr_configuration(64, 0.16), std::make_unique<FrankaRidgeback::PinocchioDynamics>(),
                                           std::make_unique<FrankaRidgeback::AssistedManipulation>(),
                                           std::make_unique<PassThrough>());
        if (t2) return 12;
    }
    std::printf("{\"cpu\": \"ok\"}\n");
    if (!gpu) return 0;

    // PinocchioDynamics through the reference's base class
    std::unique_ptr<mppi::Dynamics> d = std::make_unique<FrankaRidgeback::PinocchioDynamics>();
    mppi::VectorXd x(MPPI_FR_STATE), u(MPPI_FR_CONTROL);
    mppi_frankaridgeback_huddled(x.data());
    d->set_state(x, 0.0);
    for (int k = 0; k < 20; k++) {
        for (int i = 0; i < 12; i++) u[i] = (i >= 3 && i < 10) ? 10.0 * std::sin(0.3 * k + i) : 0.1 * std::cos(k + i);
        d->step(u, 0.01);
    }
    mppi::Ref<mppi::VectorXd> s = d->get_state();
    auto *pd = dynamic_cast<FrankaRidgeback::PinocchioDynamics *>(d.get());
    FrankaRidgeback::EndEffectorState ee = pd->get_end_effector_state();
    FrankaRidgeback::AssistedManipulation cost;
    cost.reset(0.0);
    const double wrench[6] = {20.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    pd->set_forecast([&](double, double *w) {
        std::memcpy(w, wrench, sizeof(wrench));
        return true;
    });
    mppi::VectorXd state(MPPI_FR_STATE);
    for (int i = 0; i < MPPI_FR_STATE; i++) state[i] = s[i];
    const double c = cost.get_cost(state, u, d.get(), 0.2);
    std::printf("{\"state\": [");
    for (int i = 0; i < MPPI_FR_STATE; i++) std::printf("%s%.17g", i ? ", " : "", s[i]);
    std::printf("], ");
    print_vec("ee_position", ee.position, 3);
    print_vec("ee_linear_acceleration", ee.linear_acceleration, 3);
    std::printf("\"cost\": %.17g, \"joint\": %.17g, \"workspace\": %.17g, \"trajectory\": %.17g}\n", c,
                cost.get_joint_limit_cost(), cost.get_workspace_cost(), cost.get_trajectory_cost());

    // the optimal rollout's per-term totals through get_optimal_cost() (base.cpp:140-146)
    auto traj = mppi::Trajectory::create(fr_configuration(256, 0.32), std::make_unique<FrankaRidgeback::PinocchioDynamics>(),
                                         std::make_unique<FrankaRidgeback::AssistedManipulation>());
    if (!traj) return 2;
    traj->set_noise_source(MPPI_NOISE_DEVICE_PHILOX, 0x5EED);
    std::vector<double> table(6 * traj->get_step_count(), 0.0);
    for (unsigned k = 0; k < traj->get_step_count(); k++) table[6 * k] = 20.0;
    traj->set_forecast(table);
    std::vector<double> x0(MPPI_FR_STATE);
    mppi_frankaridgeback_huddled(x0.data());
    for (int j = 0; j < 2; j++) traj->update(x0, 0.05 * j);
    const auto &oc = dynamic_cast<const FrankaRidgeback::AssistedManipulation &>(traj->get_optimal_cost());
    const double terms[7] = {oc.get_joint_limit_cost(), oc.get_self_collision_cost(), oc.get_workspace_cost(),
                             oc.get_energy_tank_cost(), oc.get_joint_velocity_cost(), oc.get_trajectory_cost(),
                             oc.get_manipulability_cost()};
    std::printf("{");
    print_vec("terms", terms, 7);
    std::printf("\"optimal_cost\": %.17g}\n", traj->get_optimal_total_cost());

    // DynamicsForecast on the trajectory's device forecast (LOCF of a constant wrench)
    FrankaRidgeback::DynamicsForecast::Configuration fc{};
    fc.time_step = 0.01;
    fc.horison = 0.2;
    fc.end_effector_wrench_forecast.type = MPPI_FORECAST_LOCF;
    fc.end_effector_wrench_forecast.locf_horison = 1.0;
    auto forecast = FrankaRidgeback::DynamicsForecast::create(fc, std::make_unique<FrankaRidgeback::PinocchioDynamics>(), *traj);
    if (!forecast) return 3;
    const double w[6] = {5.0, -2.0, 1.0, 0.0, 0.0, 0.0};
    forecast->observe_wrench(w, 0.1);
    std::vector<double> fs(MPPI_FR_STATE);
    mppi_frankaridgeback_huddled(fs.data());
    fs[12 + 4] = 0.5;
    forecast->forecast(fs, 0.1);
    const FrankaRidgeback::EndEffectorState e5 = forecast->get_end_effector_state(0.155);
    std::printf("{\"steps\": %u, ", forecast->get_steps());
    print_vec("q_last", forecast->get_joint_position(forecast->get_steps() - 1).data(), 12);
    print_vec("wrench_0", forecast->get_wrench(0).data(), 6);
    print_vec("ee5_position", e5.position, 3);
    std::printf("\"energy_last\": %.17g}\n", forecast->get_energy(forecast->get_steps() - 1));
    return 0;
}
