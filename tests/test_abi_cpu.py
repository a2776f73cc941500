"""CPU tests of the C-ABI boundary (no compute calls — there is no GPU here): the engine library
loads, exports every entry point include/mppi_amd.h declares, its structs have the header's
layout, and the host-side validation / sharding logic behaves like the reference's
Trajectory::create and ThreadPool partition."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import assistedmanipulation_amd as am
from assistedmanipulation_amd import _lib, abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "mppi_amd.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mppi_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 35
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = set(re.findall(r" T (mppi_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    assert set(names) == set(_lib.PROTOTYPES), "ctypes prototypes out of sync with the header"
    L = _lib.load()
    for n in names:
        getattr(L, n)


def test_struct_layout_matches_header(tmp_path):
    src = tmp_path / "sizes.c"
    structs = ["mppi_config", "mppi_body", "mppi_frame", "mppi_frankaridgeback_desc", "mppi_point_mass_desc",
               "mppi_dynamics_desc", "mppi_quadratic", "mppi_barrier", "mppi_assisted_manipulation_desc",
               "mppi_quadratic_cost_desc", "mppi_track_point_desc", "mppi_cost_desc"]
    body = "\n".join('printf("%s %%zu\\n", sizeof(%s));' % (s, s) for s in structs)
    body += '\nprintf("off_has_forecast %zu\\n", offsetof(mppi_assisted_manipulation_desc, has_forecast));'
    body += '\nprintf("off_threads %zu\\n", offsetof(mppi_config, threads));'
    body += '\nprintf("off_track_point %zu\\n", offsetof(mppi_cost_desc, track_point));'
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mppi_amd.h"\nint main(void){%s return 0;}\n' % body)
    exe = tmp_path / "sizes"
    subprocess.check_call(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)])
    got = dict(line.split() for line in subprocess.check_output([str(exe)]).decode().split("\n") if line)
    for s in structs:
        assert int(got[s]) == C.sizeof(getattr(abi, s)), s
    assert int(got["off_has_forecast"]) == abi.mppi_assisted_manipulation_desc.has_forecast.offset
    assert int(got["off_threads"]) == abi.mppi_config.threads.offset
    assert int(got["off_track_point"]) == abi.mppi_cost_desc.track_point.offset


def test_abi_version_and_defaults():
    L = _lib.load()
    assert L.mppi_abi_version() == 5   # 2: mppi_cost_desc.track_point; 3: device forecast; 4: dynamics object, terms;
    # 5: mppi_device_costs_count, mppi_update_last, MPPI_INFO_GRAPH_* / UPDATE_COUNT
    m = am.FrankaRidgebackDynamics().model
    assert m.nbodies == 12
    assert [m.bodies[i].parent for i in range(12)] == [-1, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 9]
    assert abs(m.bodies[2].mass - 169.235) < 1e-9          # pivot + base + chassis + imu + link0
    assert abs(m.bodies[9].mass - 1.27) < 1e-12            # link7 + hand
    assert m.end_effector.parent == 9 and abs(m.end_effector.translation[2] - 0.202) < 1e-15
    assert m.arm_mount.parent == 2
    np.testing.assert_allclose(list(m.arm_mount.translation), [0.295, 0.005, 0.725], atol=1e-15)
    c = am.AssistedManipulation().configuration
    assert c.enable_energy_limit == 0 and c.has_forecast == 1
    assert c.upper_joint_limit[8].bound == 4.53785 and c.velocity_cost[0].quadratic_cost == 1000.0
    t = am.TrackPoint().configuration   # track_point.hpp:72-107
    assert list(t.point) == [1.0, 1.0, 1.0] and t.enable_joint_limits == 1 and t.enable_reach_limits == 0
    assert t.lower_joint_limit[4].scale == 50.0 and t.maximum_reach_limit.bound == 0.8


@pytest.mark.parametrize("R,world", [(4098, 1), (4098, 2), (32770, 8), (65538, 8), (130, 3), (7, 3)])
def test_shard_range_partitions_like_the_thread_pool(R, world):
    spans = [am.shard_range(R, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == R
    for (b0, e0), (b1, e1) in zip(spans, spans[1:]):
        assert e0 == b1
    sizes = [e - b for b, e in spans]
    assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)
    assert spans[0][1] >= 2   # rollouts 0 (zero noise) and 1 (-U*) live on rank 0


def test_shard_range_rejects_bad_input():
    for args in ((10, 0, 0), (10, 2, 2), (3, 2, 0)):
        with pytest.raises(am.EngineError):
            am.shard_range(*args)


def _create(conf=None, dyn=None, cost=None):
    conf = conf or am.frankaridgeback_configuration(rollouts=32)
    return am.Trajectory.create(conf, dyn or am.FrankaRidgebackDynamics(), cost or am.AssistedManipulation())


def _err():
    return _lib.load().mppi_last_error(None).decode()


def test_create_validation_matches_reference_messages():
    """Trajectory::create's checks (mppi.cpp:17-69) run before any device call."""
    assert _create(dyn=am.PointMassDynamics()) is None
    assert "control dof 3 != cost control dof 12" in _err()
    bad = am.frankaridgeback_configuration(rollouts=32)
    bad.rollouts = 0
    assert _create(bad) is None and "rollouts must be greater than zero" in _err()
    bad = am.frankaridgeback_configuration(rollouts=32)
    bad.keep_best_rollouts = -1
    assert _create(bad) is None and "cannot be less than zero" in _err()
    bad = am.frankaridgeback_configuration(rollouts=32)
    bad.threads = 0
    assert _create(bad) is None and "threads must be positive" in _err()
    bad = am.frankaridgeback_configuration(rollouts=8, keep_best_rollouts=20)
    assert _create(bad) is None and "keep_best_rollouts > rollouts" in _err()


def test_create_rejects_unsupported_models():
    cost = am.AssistedManipulation()
    cost.configuration.enable_energy_limit = 1   # supported: validation passes it through
    if _create(cost=cost) is None:
        assert "enable_energy_limit" not in _err()
    dyn = am.FrankaRidgebackDynamics()
    dyn.model.bodies[11].parent = 10
    assert _create(dyn=dyn) is None and "topology" in _err()
    dyn = am.FrankaRidgebackDynamics()
    dyn.model.bodies[1].rotation[1] = 1e-3   # the solve takes the base joints' axes as world x / y
    assert _create(dyn=dyn) is None and "must be unrotated" in _err()
    for i in (2, 3):   # the FK scan's planar last level (fr_coop.hip scan_level_planar8)
        dyn = am.FrankaRidgebackDynamics()
        dyn.model.bodies[i].rotation[5] = 1e-3
        assert _create(dyn=dyn) is None and "rotation about z" in _err()
    dyn = am.FrankaRidgebackDynamics()   # a rotation about z is accepted
    c, s = np.cos(0.3), np.sin(0.3)
    for k, v in enumerate((c, -s, 0.0, s, c, 0.0, 0.0, 0.0, 1.0)):
        dyn.model.bodies[3].rotation[k] = v
    assert "rotation about z" not in (_err() if _create(dyn=dyn) is None else "")
