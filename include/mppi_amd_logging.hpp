// mppi_amd_logging.hpp — the reference's MPPI CSV logger (src/logging/mppi.{hpp,cpp},
// logging/csv.hpp, logging/file.hpp) over the drop-in mppi::Trajectory of mppi_amd.hpp
// (observability parity).  Same class name, Configuration fields, file names,
// headers, row layout and number formatting (a default-formatted std::fstream), so the
// reference's analysis.py reads GPU runs unchanged:
//
//   costs.csv, weights.csv        update, time, rollout1..rolloutR
//   gradient.csv,                 update, time, control1..controlC   one row per horizon step,
//   optimal_rollout.csv                                             time = t + k dt
//   optimal_cost.csv              update, time, cost
//   update.csv                    update, time, update_duration
#pragma once

#include <cstddef>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <limits>
#include <memory>
#include <string>
#include <vector>

#include "mppi_amd.hpp"

namespace logger {

// logging/csv.hpp: header and rows joined by ", ", one row per write.
class CSV {
public:
    using Header = std::vector<std::string>;
    struct Configuration {
        std::filesystem::path path;
        Header header;
    };

    static std::unique_ptr<CSV> create(const Configuration &configuration)
    {
        const std::filesystem::path parent = configuration.path.parent_path();
        if (!parent.empty() && !std::filesystem::exists(parent)) {   // File::create (file.hpp)
            std::error_code code;
            if (!std::filesystem::create_directories(parent, code)) {
                std::cerr << "failed to create log file " << configuration.path << ". " << code.message() << std::endl;
                return nullptr;
            }
        }
        std::unique_ptr<CSV> csv(new CSV());
        csv->m_stream.open(configuration.path, std::ios::out);
        if (!csv->m_stream.is_open()) {
            std::cerr << "failed to open log file " << configuration.path << std::endl;
            std::cerr << "failed to create csv log file" << std::endl;
            return nullptr;
        }
        if (!configuration.header.empty()) {
            csv->m_stream << configuration.header[0];
            for (std::size_t i = 1; i < configuration.header.size(); i++) csv->m_stream << ", " << configuration.header[i];
            csv->m_stream << '\n';
        }
        return csv;
    }

    // update, time, then either one scalar or a sequence of values
    template <class Index, class Time>
    void write(Index update, Time time, double value)
    {
        m_stream << update << ", " << time << ", " << value << '\n';
    }
    template <class Index, class Time>
    void write(Index update, Time time, const double *values, std::size_t n)
    {
        m_stream << update << ", " << time;
        if (n) {
            m_stream << ", " << values[0];
            for (std::size_t i = 1; i < n; i++) m_stream << ", " << values[i];
        }
        m_stream << '\n';
    }
    void flush() { m_stream.flush(); }
    ~CSV()
    {
        m_stream.flush();
        m_stream.close();
    }

private:
    CSV() = default;
    std::fstream m_stream;
};

// logging/mppi.{hpp,cpp}
class MPPI {
public:
    struct Configuration {
        std::filesystem::path folder;
        unsigned int state_dof;
        unsigned int control_dof;
        std::size_t rollouts;
        bool log_costs = true;
        bool log_weights = true;
        bool log_gradient = true;
        bool log_optimal_rollout = true;
        bool log_optimal_cost = true;
        bool log_update = true;
    };

    static std::unique_ptr<MPPI> create(const Configuration &configuration)
    {
        CSV::Header control, rollouts;
        for (unsigned int i = 1; i < configuration.control_dof + 1; i++) control.push_back("control" + std::to_string(i));
        for (std::size_t i = 1; i < configuration.rollouts + 1; i++) rollouts.push_back("rollout" + std::to_string(i));
        auto header = [](const CSV::Header &tail) {
            CSV::Header h{"update", "time"};
            h.insert(h.end(), tail.begin(), tail.end());
            return h;
        };
        std::unique_ptr<MPPI> mppi(new MPPI());
        const std::filesystem::path &f = configuration.folder;
        if (configuration.log_costs) mppi->m_costs = CSV::create({f / "costs.csv", header(rollouts)});
        if (configuration.log_weights) mppi->m_weights = CSV::create({f / "weights.csv", header(rollouts)});
        if (configuration.log_gradient) mppi->m_gradient = CSV::create({f / "gradient.csv", header(control)});
        if (configuration.log_optimal_rollout) mppi->m_optimal_rollout = CSV::create({f / "optimal_rollout.csv", header(control)});
        if (configuration.log_optimal_cost) mppi->m_optimal_cost = CSV::create({f / "optimal_cost.csv", header({"cost"})});
        if (configuration.log_update) mppi->m_update = CSV::create({f / "update.csv", header({"update_duration"})});
        const bool error = (configuration.log_costs && !mppi->m_costs) || (configuration.log_weights && !mppi->m_weights) ||
                           (configuration.log_gradient && !mppi->m_gradient) ||
                           (configuration.log_optimal_rollout && !mppi->m_optimal_rollout) ||
                           (configuration.log_optimal_cost && !mppi->m_optimal_cost) || (configuration.log_update && !mppi->m_update);
        if (error) {
            std::cerr << "failed to create csv logger" << std::endl;
            return nullptr;
        }
        mppi->m_last_update = std::numeric_limits<double>::min();   // as the reference (mppi.cpp:81)
        return mppi;
    }

    // MPPI::log (logging/mppi.cpp:84-136): once per update
    void log(const mppi::Trajectory &trajectory)
    {
        const double time = trajectory.get_update_last();
        if (time == m_last_update) return;
        const double step = trajectory.get_time_step();
        const unsigned int steps = trajectory.get_step_count();
        const std::size_t iteration = trajectory.get_update_count();
        const std::size_t C = trajectory.get_control_dof();
        if (m_update) m_update->write(iteration, time, trajectory.get_update_duration());
        m_time.resize(steps);
        for (unsigned int i = 0; i < steps; ++i) m_time[i] = time + i * step;
        if (m_costs) {
            const std::vector<double> costs = trajectory.get_costs();
            m_costs->write(iteration, time, costs.data(), costs.size());
        }
        if (m_weights) {
            const std::vector<double> weights = trajectory.get_weights();
            m_weights->write(iteration, time, weights.data(), weights.size());
        }
        if (m_gradient) {   // C x H column-major: column i is a control vector
            const std::vector<double> g = trajectory.get_gradient();
            for (unsigned int i = 0; i < steps; ++i) m_gradient->write(iteration, m_time[i], g.data() + (std::size_t)i * C, C);
        }
        if (m_optimal_rollout) {
            const std::vector<double> u = trajectory.get_optimal_rollout();
            for (unsigned int i = 0; i < steps; ++i) m_optimal_rollout->write(iteration, m_time[i], u.data() + (std::size_t)i * C, C);
        }
        if (m_optimal_cost) m_optimal_cost->write(iteration, time, trajectory.get_optimal_total_cost());
        m_last_update = time;
    }

private:
    MPPI() = default;
    std::unique_ptr<CSV> m_costs, m_weights, m_gradient, m_optimal_rollout, m_optimal_cost, m_update;
    std::vector<double> m_time;
    double m_last_update = 0.0;
};

}  // namespace logger
