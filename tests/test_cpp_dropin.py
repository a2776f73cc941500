"""The C++ drop-in header (include/mppi_amd.hpp) compiles with g++ against the engine, and on the
GPU drives the same updates as the Python API (same Philox seed -> identical results)."""
import json
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(REPO, "tests", "cpp")
EXE = os.path.join(CPP, "build", "trajectory_demo")


def build():
    subprocess.check_call(["make", "-s", "-C", CPP])
    return EXE


def test_cpp_dropin_compiles_and_validates_without_gpu():
    exe = build()
    assert os.path.exists(exe)


@pytest.mark.gpu
@pytest.mark.parametrize("objective", ["assisted_manipulation", "track_point"])
def test_cpp_dropin_matches_python_api(objective):
    import assistedmanipulation_amd as am
    from assistedmanipulation_amd import abi
    out = subprocess.check_output([build(), "256", "0.32", "3", objective], timeout=300).decode()
    lines = [json.loads(l) for l in out.strip().split("\n")]
    conf = am.frankaridgeback_configuration(rollouts=256, horison=0.32)
    cost = am.TrackPoint() if objective == "track_point" else am.AssistedManipulation()
    t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), cost)
    t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    t.set_forecast(am.constant_forecast(t.H))
    x = am.huddled_state()
    for j, rec in enumerate(lines):
        t.update(x, 0.05 * j)
        c = t.costs()
        u = t.get(0.05 * j + 0.013)
        assert rec["argmin"] == int(np.nanargmin(c))
        assert rec["min_cost"] == float(np.nanmin(c))
        assert rec["optimal_cost"] == t.get_optimal_total_cost()
        assert rec["u0"] == u[0] and rec["u3"] == u[3]
        assert rec["update_count"] == j + 1


@pytest.mark.gpu
def test_csv_logger_cpp_and_python_write_the_same_files(tmp_path):
    """logger::MPPI (include/mppi_amd_logging.hpp) and the Python
    MPPILogger write the reference's CSV layout byte-for-byte identically for the same run
    (update.csv holds wall-clock durations and is only checked for shape)."""
    import assistedmanipulation_amd as am
    from assistedmanipulation_amd import abi
    from assistedmanipulation_amd.csvlog import MPPILogger
    cdir, pdir = tmp_path / "cpp", tmp_path / "py"
    subprocess.check_output([build(), "64", "0.16", "3", "assisted_manipulation", str(cdir)], timeout=300)
    conf = am.frankaridgeback_configuration(rollouts=64, horison=0.16)
    t = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    t.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    t.set_forecast(am.constant_forecast(t.H))
    log = MPPILogger(str(pdir), control_dof=t.C, rollouts=t.get_rollout_count())
    x = am.huddled_state()
    for j in range(3):
        t.update(x, 0.05 * j)
        log.log(t)
        log.log(t)   # same update time: skipped, as in the reference
    log.close()
    for name in ("costs.csv", "weights.csv", "gradient.csv", "optimal_rollout.csv", "optimal_cost.csv"):
        assert (cdir / name).read_text() == (pdir / name).read_text(), name
    cu, pu = (cdir / "update.csv").read_text().splitlines(), (pdir / "update.csv").read_text().splitlines()
    assert cu[0] == pu[0] == "update, time, update_duration" and len(cu) == len(pu) == 4
    assert [l.split(", ")[:2] for l in cu] == [l.split(", ")[:2] for l in pu]


PLUGIN = os.path.join(CPP, "build", "plugin_surface")


def test_reference_shaped_plugins_compile_and_are_refused_without_a_descriptor():
    """Plugins written against the reference's pure virtuals (mppi.hpp:47-84, 110-144, 163-175,
    with `override`) compile against include/mppi_amd.hpp; Trajectory::create returns nullptr for
    a plugin without a device descriptor and for any filter (no CPU rollout path).  No GPU."""
    build()
    out = subprocess.run([PLUGIN], capture_output=True, timeout=120)
    assert out.returncode == 0, out.stderr.decode()
    assert json.loads(out.stdout.decode().strip().split("\n")[0]) == {"cpu": "ok"}
    err = out.stderr.decode()
    assert "device descriptor" in err and "filters are not supported" in err


@pytest.mark.gpu
def test_cpp_plugin_surface_on_the_device():
    """The C++ plugins' methods run on the device: PinocchioDynamics through mppi::Dynamics*,
    AssistedManipulation::get_cost against it, get_optimal_cost()'s per-term totals and
    DynamicsForecast::forecast equal the Python API's (same kernels, same inputs)."""
    import assistedmanipulation_amd as am
    from assistedmanipulation_amd import abi
    build()
    lines = [json.loads(l) for l in subprocess.check_output([PLUGIN, "gpu"], timeout=300).decode().strip().split("\n")]
    assert lines[0] == {"cpu": "ok"}
    d = am.PinocchioDynamicsObject.create(am.huddled_state())
    d.set_state(am.huddled_state(), 0.0)
    for k in range(20):
        u = np.array([10.0 * np.sin(0.3 * k + i) if 3 <= i < 10 else 0.1 * np.cos(k + i) for i in range(12)])
        d.step(u, 0.01)
    x = d.get_state()
    assert lines[1]["state"] == list(x)
    ee = d.get_end_effector_state()
    assert lines[1]["ee_position"] == list(ee.position)
    assert lines[1]["ee_linear_acceleration"] == list(ee.linear_acceleration)
    c, t = am.evaluate_cost(am.AssistedManipulation(), d, x, u, np.array([20.0, 0, 0, 0, 0, 0]))
    assert lines[1]["cost"] == c and lines[1]["joint"] == t[0] and lines[1]["workspace"] == t[2]
    assert lines[1]["trajectory"] == t[5]
    conf = am.frankaridgeback_configuration(rollouts=256, horison=0.32)
    traj = am.Trajectory.create(conf, am.FrankaRidgebackDynamics(), am.AssistedManipulation())
    traj.set_noise_source(abi.MPPI_NOISE_DEVICE_PHILOX, seed=0x5EED)
    traj.set_forecast(am.constant_forecast(traj.H))
    for j in range(2):
        traj.update(am.huddled_state(), 0.05 * j)
    assert lines[2]["terms"] == list(traj.get_optimal_terms())
    assert lines[2]["optimal_cost"] == traj.get_optimal_total_cost()
    traj.attach_forecast(am.locf_forecast_configuration(horison=1.0))
    traj.observe_wrench(np.array([5.0, -2.0, 1.0, 0, 0, 0]), 0.1)
    df = am.DynamicsForecast(0.01, 0.2, am.PinocchioDynamicsObject.create(am.huddled_state()), traj)
    fs = am.huddled_state()
    fs[12 + 4] = 0.5
    df.forecast(fs, 0.1)
    assert lines[3]["steps"] == df.steps == 20
    assert lines[3]["q_last"] == list(df.get_joint_position()[-1])
    assert lines[3]["wrench_0"] == list(df.get_wrench_trajectory()[0])
    assert lines[3]["ee5_position"] == list(df.get_end_effector_state(0.155).position)
    assert lines[3]["energy_last"] == df.get_energy_trajectory()[-1]
