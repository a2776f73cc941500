"""The Python MPPI CSV logger (assistedmanipulation_amd/csvlog.py) against the reference's layout
(logging/mppi.cpp:9-136, csv.hpp) on a hand-built trajectory stand-in: no GPU needed."""
import numpy as np

from assistedmanipulation_amd.csvlog import MPPILogger, _fmt


class _Traj:
    def __init__(self, t, n):
        self.t, self.n = t, n

    def get_update_last(self):
        return self.t

    def get_time_step(self):
        return 0.01

    def get_step_count(self):
        return 2

    def get_update_count(self):
        return self.n

    def get_update_duration(self):
        return 0.00125

    def costs(self):
        return np.array([2e11, 1.5, float("nan")])

    def get_weights(self):
        return np.array([0.0, 1.0, 0.0])

    def get_gradient(self):
        return np.array([[0.1, -2.0], [3e-7, 4.0]])

    def get_optimal_rollout(self):
        return np.array([[1.0, 2.0], [3.0, 4.0]])

    def get_optimal_total_cost(self):
        return 123456789.0


def test_number_format_is_default_ostream():
    assert [_fmt(v) for v in (2e11, 1.5, 0.1, 3e-7, 123456789.0, 0.0, -2.0, 1e10, 0.05)] == \
        ["2e+11", "1.5", "0.1", "3e-07", "1.23457e+08", "0", "-2", "1e+10", "0.05"]
    assert _fmt(float("nan")) == "nan" and _fmt(float("inf")) == "inf"


def test_files_headers_and_rows(tmp_path):
    log = MPPILogger(str(tmp_path), control_dof=2, rollouts=3)
    log.log(_Traj(0.05, 1))
    log.log(_Traj(0.05, 1))   # repeated update time: skipped (mppi.cpp:87-88)
    log.close()
    read = lambda n: (tmp_path / n).read_text()  # noqa: E731
    assert read("costs.csv") == "update, time, rollout1, rollout2, rollout3\n1, 0.05, 2e+11, 1.5, nan\n"
    assert read("weights.csv") == "update, time, rollout1, rollout2, rollout3\n1, 0.05, 0, 1, 0\n"
    assert read("gradient.csv") == "update, time, control1, control2\n1, 0.05, 0.1, -2\n1, 0.06, 3e-07, 4\n"
    assert read("optimal_rollout.csv") == "update, time, control1, control2\n1, 0.05, 1, 2\n1, 0.06, 3, 4\n"
    assert read("optimal_cost.csv") == "update, time, cost\n1, 0.05, 1.23457e+08\n"
    assert read("update.csv") == "update, time, update_duration\n1, 0.05, 0.00125\n"
