"""The reference's MPPI CSV logger (src/logging/mppi.{hpp,cpp}, csv.hpp, file.hpp) for the Python
front end: same file names, headers, row layout and number formatting as a default-formatted
std::fstream (6 significant digits, "%.6g"), so the reference's analysis.py reads GPU runs and
the output is byte-identical to include/mppi_amd_logging.hpp's logger::MPPI.
"""
import os
import sys

_DBL_MIN = sys.float_info.min   # std::numeric_limits<double>::min() (logging/mppi.cpp:81)


def _fmt(v):
    """operator<<(std::ostream&, double) with the default flags and precision 6."""
    v = float(v)
    if v != v:
        return "-nan" if str(v).startswith("-") else "nan"
    if v in (float("inf"), float("-inf")):
        return "inf" if v > 0 else "-inf"
    return "%.6g" % v


class _CSV:
    def __init__(self, path, header):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        self._f = open(path, "w")
        if header:
            self._f.write(", ".join(header) + "\n")

    def write(self, update, time, values):
        row = [str(int(update)), _fmt(time)] + [_fmt(v) for v in values]
        self._f.write(", ".join(row) + "\n")

    def close(self):
        self._f.flush()
        self._f.close()


class MPPILogger:
    """logger::MPPI: `log(trajectory)` once per update (repeated times are skipped)."""

    def __init__(self, folder, control_dof, rollouts, log_costs=True, log_weights=True, log_gradient=True,
                 log_optimal_rollout=True, log_optimal_cost=True, log_update=True):
        control = ["control%d" % i for i in range(1, control_dof + 1)]
        rolls = ["rollout%d" % i for i in range(1, rollouts + 1)]
        p = lambda name: os.path.join(folder, name)  # noqa: E731
        self._costs = _CSV(p("costs.csv"), ["update", "time"] + rolls) if log_costs else None
        self._weights = _CSV(p("weights.csv"), ["update", "time"] + rolls) if log_weights else None
        self._gradient = _CSV(p("gradient.csv"), ["update", "time"] + control) if log_gradient else None
        self._optimal_rollout = _CSV(p("optimal_rollout.csv"), ["update", "time"] + control) if log_optimal_rollout else None
        self._optimal_cost = _CSV(p("optimal_cost.csv"), ["update", "time", "cost"]) if log_optimal_cost else None
        self._update = _CSV(p("update.csv"), ["update", "time", "update_duration"]) if log_update else None
        self._last = _DBL_MIN

    def log(self, trajectory):
        time = trajectory.get_update_last()
        if time == self._last:
            return
        step, steps = trajectory.get_time_step(), trajectory.get_step_count()
        it = trajectory.get_update_count()
        if self._update:
            self._update.write(it, time, [trajectory.get_update_duration()])
        times = [time + i * step for i in range(steps)]
        if self._costs:
            self._costs.write(it, time, trajectory.costs())
        if self._weights:
            self._weights.write(it, time, trajectory.get_weights())
        if self._gradient:
            g = trajectory.get_gradient()   # (H, C): row k = column k of the C x H gradient
            for i in range(steps):
                self._gradient.write(it, times[i], g[i])
        if self._optimal_rollout:
            u = trajectory.get_optimal_rollout()
            for i in range(steps):
                self._optimal_rollout.write(it, times[i], u[i])
        if self._optimal_cost:
            self._optimal_cost.write(it, time, [trajectory.get_optimal_total_cost()])
        self._last = time

    def close(self):
        for f in (self._costs, self._weights, self._gradient, self._optimal_rollout, self._optimal_cost, self._update):
            if f:
                f.close()
