// Drives the engine through the C++ drop-in (include/mppi_amd.hpp) the way the reference's
// FrankaRidgeback::Actor drives mppi::Trajectory (actor.cpp:96-101, 166-203):
// create -> per control period: set_forecast, update(state, t), get(control, t).
// Prints one JSON object per update.
// Usage: trajectory_demo [rollouts] [horison] [updates] [assisted_manipulation|track_point] [log folder]
// With a log folder, logger::MPPI (mppi_amd_logging.hpp) writes the reference's CSV files there.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mppi_amd.hpp"
#include "mppi_amd_logging.hpp"

int main(int argc, char **argv)
{
    const long rollouts = argc > 1 ? std::atol(argv[1]) : 128;
    const double horison = argc > 2 ? std::atof(argv[2]) : 0.32;
    const int updates = argc > 3 ? std::atoi(argv[3]) : 3;
    const bool track_point = argc > 4 && std::strcmp(argv[4], "track_point") == 0;
    auto objective = [&]() -> std::unique_ptr<mppi::Cost> {
        if (track_point) return FrankaRidgeback::TrackPoint::create(FrankaRidgeback::TrackPoint::DEFAULT_CONFIGURATION);
        return std::make_unique<FrankaRidgeback::AssistedManipulation>();
    };

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

    {   // the reference's create() validation: nullptr + message
        mppi::Configuration bad = c;
        bad.rollouts = 0;
        auto t = mppi::Trajectory::create(bad, std::make_unique<FrankaRidgeback::PinocchioDynamics>(),
                                          std::make_unique<FrankaRidgeback::AssistedManipulation>());
        if (t) { std::printf("{\"error\": \"invalid configuration accepted\"}\n"); return 1; }
    }
    auto traj = mppi::Trajectory::create(c, std::make_unique<FrankaRidgeback::PinocchioDynamics>(), objective());
    if (!traj) return 2;
    std::unique_ptr<logger::MPPI> log;
    if (argc > 5) {   // base.cpp:49-61: the logger sized to the controller's rollout count
        logger::MPPI::Configuration lc;
        lc.folder = argv[5];
        lc.state_dof = MPPI_FR_STATE;
        lc.control_dof = MPPI_FR_CONTROL;
        lc.rollouts = traj->get_rollout_count();
        log = logger::MPPI::create(lc);
        if (!log) return 3;
    }
    traj->set_noise_source(MPPI_NOISE_DEVICE_PHILOX, 0x5EED);
    std::vector<double> forecast(6 * traj->get_step_count(), 0.0);
    for (unsigned k = 0; k < traj->get_step_count(); k++) forecast[6 * k] = 20.0;
    traj->set_forecast(forecast);
    std::vector<double> state = c.initial_state, control(12);
    for (int j = 0; j < updates; j++) {
        const double t = 0.05 * j;
        traj->update(state, t);
        traj->get(control, t + 0.013);
        if (log) log->log(*traj);
        std::vector<double> costs = traj->get_costs();
        long best = 0;
        for (long r = 1; r < (long)costs.size(); r++)
            if (costs[r] < costs[best]) best = r;
        std::printf("{\"update\": %d, \"argmin\": %ld, \"min_cost\": %.17g, \"optimal_cost\": %.17g, "
                    "\"u0\": %.17g, \"u3\": %.17g, \"update_count\": %zu}\n",
                    j, best, costs[best], traj->get_optimal_total_cost(), control[0], control[3], traj->get_update_count());
    }
    return 0;
}
