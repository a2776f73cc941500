#!/usr/bin/env python3
"""Generate the golden vectors that pin the CPU oracle (run in the build container, where the
reference tree is mounted; the outputs in tests/golden/*.npz are committed and used offline).

This is an INDEPENDENT float64 numpy restatement, deliberately built differently from
oracle/mppi_oracle.cpp so that agreement means something:

  * robot model: robot.urdf parsed again here, links kept separate (no fixed-joint inertia
    merging), rpy -> matrix by direct Rz Ry Rx products (not the urdfdom quaternion path);
  * dynamics: mass matrix by composite Jacobians, M = sum_l m_l Jv_l^T Jv_l + Jw_l^T I_l Jw_l
    over every link with mass, then a = solve(M, tau_u) (LU) — instead of RNEA + ABA;
  * WORLD Jacobian / frame velocity: per-joint p x a, and checked against finite differences of
    the end-effector pose (v_O = v_point - omega x p);
  * cost and the MPPI update loop (sample / rollout / optimise / SG / clamp / filter) rewritten
    in plain Python from the reference sources (mppi.cpp, assisted_manipulation.cpp, cost.hpp,
    filter.cpp, gram_savitzky_golay.cpp).

The reference itself cannot be built here (Eigen3 + Pinocchio are absent), so
the Pinocchio boundary is pinned by this model plus physics identities (tests/test_oracle_cpu.py).
"""
import math
import os
import sys
import xml.etree.ElementTree as ET

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
URDF = "/root/reference/src/frankaridgeback/model/robot.urdf"


# ------------------------------------------------------------------------------------------
# robot model (links unmerged)
# ------------------------------------------------------------------------------------------
def rpy_matrix(r, p, y):
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1.0]])
    Ry = np.array([[cp, 0, sp], [0, 1.0, 0], [-sp, 0, cp]])
    Rx = np.array([[1.0, 0, 0], [0, cr, -sr], [0, sr, cr]])
    return Rz @ Ry @ Rx


def origin_T(el):
    T = np.eye(4)
    o = el.find("origin") if el is not None else None
    if o is not None:
        xyz = [float(v) for v in o.get("xyz", "0 0 0").split()]
        rpy = [float(v) for v in o.get("rpy", "0 0 0").split()]
        T[:3, :3] = rpy_matrix(*rpy)
        T[:3, 3] = xyz
    return T


class Robot:
    def __init__(self, path=URDF):
        root = ET.parse(path).getroot()
        self.links = {l.get("name"): l for l in root.findall("link")}
        self.joints = {j.get("name"): j for j in root.findall("joint")}
        self.parent_joint = {}
        for name, j in self.joints.items():
            self.parent_joint[j.find("child").get("link")] = name
        # moving joints in DoF order (frankaridgeback/dof.hpp)
        self.dof = ["x_base_joint", "y_base_joint", "pivot_joint"] + ["panda_joint%d" % i for i in range(1, 8)] + \
                   ["panda_finger_joint1", "panda_finger_joint2"]
        self.root = [l for l in self.links if l not in self.parent_joint][0]
        self.inertial = {}
        for name, l in self.links.items():
            i = l.find("inertial")
            if i is None:
                continue
            m = float(i.find("mass").get("value"))
            if m == 0.0:
                continue
            T = origin_T(i)
            e = i.find("inertia")
            g = lambda k: float(e.get(k, "0"))
            I = np.array([[g("ixx"), g("ixy"), g("ixz")], [g("ixy"), g("iyy"), g("iyz")], [g("ixz"), g("iyz"), g("izz")]])
            self.inertial[name] = (m, T[:3, 3].copy(), T[:3, :3] @ I @ T[:3, :3].T)

    def chain(self, link):
        """joints from the root to `link`."""
        out = []
        while link in self.parent_joint:
            j = self.parent_joint[link]
            out.append(j)
            link = self.joints[j].find("parent").get("link")
        return out[::-1]

    def link_pose(self, q, link):
        """World pose of a link frame, and the world axis/origin of every moving joint on the way."""
        T = np.eye(4)
        axes = {}
        for jn in self.chain(link):
            j = self.joints[jn]
            T = T @ origin_T(j)
            t = j.get("type")
            if t in ("revolute", "prismatic"):
                a = np.array([float(v) for v in j.find("axis").get("xyz").split()])
                qi = q[self.dof.index(jn)]
                axes[jn] = (T[:3, :3] @ a, T[:3, 3].copy(), t)
                M = np.eye(4)
                if t == "revolute":
                    a = a / np.linalg.norm(a)
                    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
                    M[:3, :3] = np.eye(3) + math.sin(qi) * K + (1 - math.cos(qi)) * K @ K
                else:
                    M[:3, 3] = a * qi
                T = T @ M
        return T, axes

    def mass_matrix(self, q):
        n = len(self.dof)
        M = np.zeros((n, n))
        for link, (m, c_local, I_local) in self.inertial.items():
            T, axes = self.link_pose(q, link)
            R, p = T[:3, :3], T[:3, 3]
            c = p + R @ c_local
            Iw = R @ I_local @ R.T
            Jv = np.zeros((3, n))
            Jw = np.zeros((3, n))
            for jn, (a, o, t) in axes.items():
                k = self.dof.index(jn)
                if t == "revolute":
                    Jv[:, k] = np.cross(a, c - o)
                    Jw[:, k] = a
                else:
                    Jv[:, k] = a
            M += m * Jv.T @ Jv + Jw.T @ Iw @ Jw
        return M

    def link_pose_any(self, q, link):
        """link_pose for real or complex q (np.sin / np.cos): the complex-step derivatives of
        nle() differentiate the mass matrix through it."""
        dtype = np.complex128 if np.iscomplexobj(q) else np.float64
        T = np.eye(4, dtype=dtype)
        axes = {}
        for jn in self.chain(link):
            j = self.joints[jn]
            T = T @ origin_T(j)
            t = j.get("type")
            if t in ("revolute", "prismatic"):
                a = np.array([float(v) for v in j.find("axis").get("xyz").split()])
                qi = q[self.dof.index(jn)]
                axes[jn] = (T[:3, :3] @ a, T[:3, 3].copy(), t)
                M = np.eye(4, dtype=dtype)
                if t == "revolute":
                    a = a / np.linalg.norm(a)
                    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
                    M[:3, :3] = np.eye(3) + np.sin(qi) * K + (1 - np.cos(qi)) * K @ K
                else:
                    M[:3, 3] = a * qi
                T = T @ M
        return T, axes

    def link_jacobians(self, q, link):
        """World com, linear and angular Jacobians of a link's centre of mass (real or complex q)."""
        m, c_local, I_local = self.inertial[link]
        T, axes = self.link_pose_any(q, link)
        R, p = T[:3, :3], T[:3, 3]
        c = p + R @ c_local
        n = len(self.dof)
        Jv = np.zeros((3, n), dtype=T.dtype)
        Jw = np.zeros((3, n), dtype=T.dtype)
        for jn, (a, o, t) in axes.items():
            k = self.dof.index(jn)
            if t == "revolute":
                Jv[:, k] = np.cross(a, c - o)
                Jw[:, k] = a
            else:
                Jv[:, k] = a
        return R, c, Jv, Jw

    def mass_matrix_any(self, q):
        n = len(self.dof)
        M = np.zeros((n, n), dtype=np.complex128 if np.iscomplexobj(q) else np.float64)
        for link, (m, c_local, I_local) in self.inertial.items():
            R, c, Jv, Jw = self.link_jacobians(q, link)
            Iw = R @ I_local @ R.T
            M += m * Jv.T @ Jv + Jw.T @ Iw @ Jw
        return M

    def nle(self, q, v, g=9.81, h=1e-20):
        """Coriolis/centrifugal + gravity torques from the Lagrangian, independent of RNEA:
        g(q) = sum_l m_l Jv_l^T (0, 0, g) and C(q, v) v = Mdot v - 1/2 d(v^T M v)/dq, with Mdot and
        dM/dq_i by complex-step differentiation of the composite-Jacobian mass matrix (exact to
        rounding: no subtractive cancellation)."""
        n = len(self.dof)
        grav = np.zeros(n)
        for link, (m, c_local, I_local) in self.inertial.items():
            R, c, Jv, Jw = self.link_jacobians(q, link)
            grav += m * (Jv.T @ np.array([0.0, 0.0, g]))
        Mdot = self.mass_matrix_any(q + 1j * h * v).imag / h
        dT = np.array([v @ (self.mass_matrix_any(q + 1j * h * np.eye(n)[i]).imag / h) @ v for i in range(n)])
        return Mdot @ v - 0.5 * dT + grav

    def frame(self, q, link):
        T, axes = self.link_pose(q, link)
        return T

    def world_jacobian(self, q, link):
        """Spatial (WORLD, at the world origin) Jacobian columns of the joints supporting link."""
        _, axes = self.link_pose(q, link)
        J = np.zeros((6, len(self.dof)))
        for jn, (a, o, t) in axes.items():
            k = self.dof.index(jn)
            if t == "revolute":
                J[:3, k] = np.cross(o, a)
                J[3:, k] = a
            else:
                J[:3, k] = a
        return J


def world_jacobian_any(rob, q, link):
    """world_jacobian for real or complex q (link_pose_any)."""
    _, axes = rob.link_pose_any(q, link)
    J = np.zeros((6, len(rob.dof)), dtype=np.complex128 if np.iscomplexobj(q) else np.float64)
    for jn, (a, o, t) in axes.items():
        k = rob.dof.index(jn)
        if t == "revolute":
            J[:3, k] = np.cross(o, a)
            J[3:, k] = a
        else:
            J[:3, k] = a
    return J


def ee_acceleration(rob, q, v, a, link, h=1e-20):
    """Spatial acceleration at the world origin (what Pinocchio's getFrameAcceleration(WORLD)
    returns: the time derivative of the WORLD spatial velocity J(q) v) along q(t) = q + v t,
    v(t) = v + a t, by complex-step differentiation in t: Im(J(q + i h v)(v + i h a)) / h =
    Jdot v + J a, exact to rounding, no RNEA."""
    return (world_jacobian_any(rob, q + 1j * h * v, link) @ (v + 1j * h * a)).imag / h


def quaternion_xyzw(R):
    """A unit quaternion (x, y, z, w) of R with w >= 0 (Shoemake's, independent of Eigen's branch
    order; compared up to sign)."""
    w = math.sqrt(max(0.0, 1.0 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    x = math.sqrt(max(0.0, 1.0 + R[0, 0] - R[1, 1] - R[2, 2])) / 2
    y = math.sqrt(max(0.0, 1.0 - R[0, 0] + R[1, 1] - R[2, 2])) / 2
    z = math.sqrt(max(0.0, 1.0 - R[0, 0] - R[1, 1] + R[2, 2])) / 2
    x = math.copysign(x, R[2, 1] - R[1, 2])
    y = math.copysign(y, R[0, 2] - R[2, 0])
    z = math.copysign(z, R[1, 0] - R[0, 1])
    return np.array([x, y, z, w])


def gen_end_effector(rob, n=24, seed=7):
    """EndEffectorState fixtures beyond kinematics.npz: the EE orientation (matrix and quaternion)
    and its WORLD spatial acceleration, at random (q, v) with qdd = M^-1 tau."""
    rng = np.random.default_rng(seed)
    x0 = huddled()
    qs, vs, taus, outs = [], [], [], []
    for i in range(n):
        q = x0[:12] + rng.normal(0, 0.6, 12) * (1 if i else 0)
        q[10:] = np.abs(q[10:]) * 0.05 + 0.01
        v = rng.normal(0, 1.0, 12)
        tau = rng.normal(0, 5.0, 12)
        a = np.linalg.solve(rob.mass_matrix(q), tau)
        T = rob.frame(q, EE_LINK)
        R = T[:3, :3]
        A = ee_acceleration(rob, q, v, a, EE_LINK)
        qs.append(q); vs.append(v); taus.append(tau)
        outs.append(np.concatenate([R.reshape(-1), quaternion_xyzw(R), A, a]))
    return np.array(qs), np.array(vs), np.array(taus), np.array(outs)


def fd_world_velocity(rob, q, v, link, h=1e-6):
    """Spatial velocity at the world origin from finite differences of the link pose."""
    T1 = rob.frame(q - h * v, link)
    T2 = rob.frame(q + h * v, link)
    T0 = rob.frame(q, link)
    vp = (T2[:3, 3] - T1[:3, 3]) / (2 * h)
    dR = (T2[:3, :3] - T1[:3, :3]) / (2 * h)
    W = dR @ T0[:3, :3].T
    w = np.array([W[2, 1], W[0, 2], W[1, 0]])
    return np.concatenate([vp - np.cross(w, T0[:3, 3]), w])


# ------------------------------------------------------------------------------------------
# dynamics step + cost (pinocchio_dynamics.cpp:226-260, assisted_manipulation.cpp)
# ------------------------------------------------------------------------------------------
EE_LINK, AM_LINK = "panda_grasp", "franka_mount_link"


def kin(rob, q, v):
    ee = rob.frame(q, EE_LINK)[:3, 3]
    am = rob.frame(q, AM_LINK)[:3, 3]
    J = rob.world_jacobian(q, EE_LINK)
    vee = J @ v
    J = J.copy()
    c, s = math.cos(q[2]), math.sin(q[2])
    J[:3, :3] = [[c, -s, 0], [s, c, 0], [0, 0, 1]]
    return dict(ee=ee, am=am, J=J, vee=vee)


def left(bound, scale, v, mx=1e10):
    if v <= bound:
        return mx + scale * (bound - v) ** 2
    return min(scale / (v - bound), mx)


def right(bound, scale, v, mx=1e10):
    if v >= bound:
        return mx + scale * (v - bound) ** 2
    return min(scale / (bound - v), mx)


LOWER = [(-2.0, 0.0), (-2.0, 0.0), (-6.28, 0.0), (-2.8, 10.0), (-1.745, 10.0), (-2.8, 10.0), (-3.0718, 10.0),
         (-2.7925, 10.0), (0.349, 10.0), (-2.967, 10.0), (0.0, 0.0), (0.0, 0.0)]
UPPER = [(2.0, 0.0), (2.0, 0.0), (6.28, 0.0), (2.8, 10.0), (1.745, 10.0), (2.8, 10.0), (0.0, 10.0), (2.7925, 10.0),
         (4.53785, 10.0), (2.967, 10.0), (0.5, 0.0), (0.5, 0.0)]
VEL = [1000.0, 1000.0, 100.0, 0.5, 1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 0.0, 0.0]
RADII = [0.75, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1]
PAIRS = [(3, l) for l in (6, 7, 8, 9, 10)] + [(4, l) for l in (6, 7, 8, 9, 10)] + [(5, l) for l in (7, 8, 9, 10)] + \
        [(6, l) for l in (8, 9, 10)] + [(7, l) for l in (9, 10)] + [(8, 10)]


def cost(x, k_cache, force, energy=False):
    q, v = x[:12], x[12:24]
    c = 0.0
    c += sum(left(*LOWER[i], q[i]) + right(*UPPER[i], q[i]) for i in range(12))
    c += sum(1e10 + (RADII[a - 3] + RADII[b - 3]) ** 2 for a, b in PAIRS)   # link positions == 0
    ee, am = k_cache["ee"], k_cache["am"]
    f = np.array([math.cos(x[2]), math.sin(x[2]), 0.0])
    robot = am + np.array([0.1 * math.cos(x[2]), 0.1 * math.sin(x[2]), 0.15])
    d = ee - robot
    ws = left(0.0, 1.0, d @ f / (f @ f)) + right(1.0, 1.0, np.linalg.norm(d))
    cosang = (d[:2] @ f[:2]) / np.linalg.norm(d[:2]) / np.linalg.norm(f[:2])
    yaw = math.acos(cosang) if -1.0 <= cosang <= 1.0 else float("nan")
    if not math.isnan(yaw):
        ws += 400.0 * yaw * yaw
    ws += left(0.0, 1.0, ee[2] - robot[2])
    c += ws
    if energy:   # energy_cost: Left(0, 10) + Right(20, 10) of the tank energy (x[30])
        c += left(0.0, 10.0, x[30]) + right(20.0, 10.0, x[30])
    c += sum(VEL[i] * v[i] ** 2 for i in range(12))
    target = np.clip(0.01 * np.asarray(force[:3]), -1.0, 1.0)
    dist = np.linalg.norm(target)
    if dist > 0.0:
        tc = 100.0 + 500.0 * dist * dist
        proj = (k_cache["vee"][:3] @ target) / (target @ target)
        proj = math.copysign(1.0, proj) * np.linalg.norm(target * proj)
        vt = min(max(math.exp(2.0 * dist) - 1.0, 0.1), 5.0)
        tc += 500.0 * (vt - proj) ** 2
        c += tc
    Ja = k_cache["J"][:3, 3:10]
    det = np.linalg.det(Ja @ Ja.T)
    vol = math.sqrt(det) if det >= 0 else float("nan")
    vol = 1e-5 if math.isnan(vol) else min(max(vol, 1e-5), 1e5)
    c += 10.0 * (1.0 / vol) ** 2
    return c


# TrackPoint (frankaridgeback/objective/track_point.cpp:10-186): every term enabled in the fixture
TP_LO = [-2.0, -2.0, -6.28, -2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973]
TP_UP = [2.0, 2.0, 6.28, 2.8973, 1.7628, 2.8973, 0.0698, 2.8973, 3.7525, 2.8973]
TP_POINT = np.array([0.8, 0.6, 0.9])


TP_BREACHES = [0]


def track_point_cost(x, k_cache, force):
    q = x[:12]
    ee = k_cache["ee"]
    c = 100.0 * float(np.linalg.norm(ee - TP_POINT)) ** 2
    for i in range(10):
        if q[i] < TP_LO[i]:
            c += 1000.0 + 100000.0 * (TP_LO[i] - q[i]) ** 2
            TP_BREACHES[0] += 1
        if q[i] > TP_UP[i]:
            c += 1000.0 + 100000.0 * (q[i] - TP_UP[i]) ** 2
            TP_BREACHES[0] += 1
    c += sum(left(0.0, 1.0, RADII[a - 3] + RADII[b - 3]) for a, b in PAIRS)   # link positions == 0
    robot = k_cache["am"] + np.array([0.3 * math.cos(x[2]), 0.3 * math.sin(x[2]), 0.15])
    c += right(0.8, 1.0, float(np.linalg.norm(ee - robot)))
    return c


def energy_only_cost(x, k_cache, force):
    """AssistedManipulation with only enable_energy_limit set: Left(0, 10) + Right(20, 10) of E."""
    return left(0.0, 10.0, x[30]) + right(20.0, 10.0, x[30])


def energy_rollouts(rob, seed=6, H=16):
    """Free rollouts of the tank from HUDDLED: random controls with E0 = 15 and E0 = 0.05, and two
    descents (arm torque -s g(q0) lets gravity pull the arm: negative power) that reach the
    max(0, .) clamp.  Returns E0 [n], controls [n][H][12] and E after each step [n][H]."""
    rng = np.random.default_rng(seed)
    g0 = rob.nle(huddled()[:12], np.zeros(12))
    cases = [(15.0, None), (15.0, None), (0.05, None), (0.05, None), (0.5, 0.1), (0.2, 0.3)]
    us, es, e0s = [], [], []
    for e0, s in cases:
        x = huddled()
        x[30] = e0
        if s is None:
            u = rng.standard_normal((H, 12)) * np.sqrt(VAR) * 3.0
        else:
            u = np.zeros((H, 12))
            u[:, 3:10] = -s * g0[3:10]
        E = []
        for k in range(H):
            x, _ = step(rob, x, u[k], 0.01, energy=True)
            E.append(x[30])
        us.append(u); es.append(E); e0s.append(e0)
    assert min(min(e) for e in es) == 0.0
    return np.array(us), np.array(es), np.array(e0s)


def step(rob, x, u, dt, energy=False):
    q, v = x[:12].copy(), x[12:24].copy()
    c, s = math.cos(q[2]), math.sin(q[2])
    v[0] = c * u[0] - s * u[1]
    v[1] = s * u[0] + c * u[1]
    v[2] = u[2]
    tau = np.zeros(12)
    tau[3:10] = u[3:10]
    a = np.linalg.solve(rob.mass_matrix(q), tau)
    kc = kin(rob, q, v)     # computed before integration: the one-step lag
    nle = rob.nle(q, v) if energy else None   # m_joint_torque += NLE at (q, v after the overwrite)
    v = v + a * dt
    q = q + v * dt
    xn = x.copy()
    xn[:12], xn[12:24] = q, v
    if energy:   # power = (tau_u + NLE) . v_new; EnergyTank::step (energy.hpp:19-22)
        xn[30] = max(0.0, x[30] + float((tau + nle) @ v) * dt)
    return xn, kc


def rollout(rob, x0, U, eps, dt, forecast, optimal=False, objective=None, energy=False):
    objective = objective or cost
    x = x0.copy()
    kc = kin(rob, x[:12], x[12:24])
    J = 0.0
    for k in range(U.shape[0]):
        u = U[k] + (0.0 if eps is None else eps[k])
        sc = objective(x, kc, forecast[k])
        if not optimal and math.isnan(sc):
            return float("nan")
        J += sc
        if k < U.shape[0] - 1:
            x, kc = step(rob, x, u, dt, energy)
    return J


# ------------------------------------------------------------------------------------------
# Savitzky-Golay (gram_savitzky_golay.cpp + filter.cpp)
# ------------------------------------------------------------------------------------------
def sg_weights(m, n):
    """Least-squares polynomial smoothing weights at the centre of 2m+1 points (closed form via
    a Vandermonde pseudo-inverse — a different route than the Gram-polynomial recursion)."""
    x = np.arange(-m, m + 1, dtype=np.float64)
    V = np.vander(x, n + 1, increasing=True)
    return np.linalg.pinv(V)[0]


class Window:
    def __init__(self, H, w):
        self.w, self.W = w, H + 2 * w + 1
        self.uu = [0.0] * self.W
        self.tt = [-1.0] * self.W
        self.start = w
        self.last = -1.0

    def trim(self, t):
        assert t >= self.last
        self.last = t
        ti = self.start
        for i in range(self.start):
            if self.tt[i] >= t:
                ti = i
                break
        off = ti - self.w
        self.tt = self.tt[off:] + self.tt[:off]
        self.uu = self.uu[off:] + self.uu[:off]
        if off > 0:
            self.tt[self.W - off:] = [self.tt[self.W - off - 1]] * off
            self.uu[self.W - off:] = [self.uu[self.W - off - 1]] * off
        self.start = self.w
        self.tt[self.w] = t

    def add(self, u, t):
        assert not t < self.tt[self.start]
        for i in range(self.start, self.W):
            self.uu[i], self.tt[i] = u, t
        self.start += 1

    def lower(self, t):
        lo, hi = 0, self.W
        while lo < hi:
            mid = (lo + hi) // 2
            if self.tt[mid] < t:
                lo = mid + 1
            else:
                hi = mid
        return lo


# ------------------------------------------------------------------------------------------
# mppi::Trajectory (mppi.cpp) restated in Python
# ------------------------------------------------------------------------------------------
class MPPI:
    def __init__(self, rob, S, K, H, dt, var, cmin, cmax, x0, smoothing=None, objective=None, energy=False):
        self.rob, self.S, self.K, self.H, self.dt = rob, S, K, H, dt
        self.energy = energy
        self.objective = objective or cost
        self.R = S + 2
        self.C = len(var)
        self.noise = np.zeros((self.R, H, self.C))
        self.cost = np.zeros(self.R)
        self.w = np.zeros(self.R)
        self.g = np.zeros((H, self.C))
        self.U = np.zeros((H, self.C))
        self.Us = np.zeros((H, self.C))
        self.cmin, self.cmax = np.asarray(cmin), np.asarray(cmax)
        self.last_shift = 0.0
        self.windows = [Window(H, smoothing[0]) for _ in range(self.C)] if smoothing else None
        self.sgw = sg_weights(*smoothing) if smoothing else None
        self.opt_cost = 0.0

    def draws(self, t):
        sb = int((t - self.last_shift) / self.dt)
        return (self.S - self.K) * self.H + (self.K * min(sb, self.H) if sb > 0 else 0)

    def update(self, x0, t, eps, forecast):
        it = iter(eps)
        sb = int((t - self.last_shift) / self.dt)
        if sb > 0:
            self.last_shift = t
            shifted = self.H - sb
            self.Us[:shifted] = self.U[sb:]
            self.Us[shifted:] = self.U[-1]
        order = sorted(range(2, self.R), key=lambda r: (math.isnan(self.cost[r]), 0.0 if math.isnan(self.cost[r]) else self.cost[r], r))
        keep, res = order[:self.K], order[self.K:]
        if sb > 0:
            for r in keep:
                self.noise[r, :shifted] = self.noise[r, sb:].copy()
                for k in range(shifted, self.H):
                    self.noise[r, k] = next(it)
        for r in res:
            for k in range(self.H):
                self.noise[r, k] = next(it)
        self.noise[1] = -self.U
        for r in range(self.R):
            self.cost[r] = rollout(self.rob, x0, self.Us, self.noise[r], self.dt, forecast, objective=self.objective,
                                   energy=self.energy)
        ok = ~np.isnan(self.cost)
        mn, mx = self.cost[ok].min(), self.cost[ok].max()
        if mx - mn >= 1e-6:
            lik = np.where(ok, np.exp(-10.0 * (np.where(ok, self.cost, mn) - mn) / (mx - mn)), 0.0)
            self.w = lik / lik.sum()
            self.g = np.tensordot(self.w, self.noise, axes=1)
            self.Us = self.Us + 2.0 * self.g
            if self.windows:
                for c, win in enumerate(self.windows):
                    win.trim(t)
                    for k in range(self.H):
                        win.add(self.Us[k, c], t + k * self.dt)
                    for k in range(self.H):
                        tk = t + k * self.dt
                        idx = win.lower(tk)
                        v = np.array(win.uu[idx - win.w: idx + win.w + 1])
                        r = float(self.sgw @ v)
                        self.Us[k, c] = r
                        win.uu[idx - 1] = r
            self.Us = np.maximum(np.minimum(self.Us, self.cmax), self.cmin)
        self.opt_cost = rollout(self.rob, x0, self.Us, None, self.dt, forecast, optimal=True, objective=self.objective,
                                energy=self.energy)
        self.U = self.Us.copy()


VAR = np.array([0.1, 0.1, 0.2] + [7.5] * 7 + [0.0, 0.0])
CMIN = np.array([-0.5, -0.5, -1.0] + [-100.0] * 7 + [-0.05, -0.05])
CMAX = -CMIN


class KalmanForecastNp:
    """KalmanForecast + KalmanFilter (forecast.cpp:131-367, kalman.cpp:103-152) restated with
    numpy matrices: np.linalg.inv for the gain and the horison as matrix powers F^i x (the
    reference iterates predict(false)), so it is built differently from the C++ oracle."""

    def __init__(self, order, time_step, horison, initial_state):
        self.n = n = 6 * (order + 1)
        self.order, self.dt, self.horison = order, time_step, horison
        self.steps = int(math.ceil(horison / time_step))
        F = np.zeros((n, n))
        for d in range(order + 1):
            for s in range(6):
                for i in range(order - d + 1):
                    F[d * 6 + s, d * 6 + i * 6 + s] = time_step ** i / math.factorial(i)
        self.F = F
        self.Q = self.R = np.eye(n) * 1e-8
        self.P = np.eye(n) * 1e-8
        self.x = np.zeros(n)
        self.x[:6] = initial_state
        self.xn = F @ self.x
        self.meas = np.zeros(n)
        self.last = -time_step
        self.pred = np.zeros((self.steps + 1, n))

    def observe(self, m, t):
        dt = t - self.last
        delta = (np.asarray(m) - self.meas[:6]) / dt
        for i in range(1, self.order + 1):
            nxt = (delta - self.meas[6 * i:6 * i + 6]) / dt
            self.meas[6 * i:6 * i + 6] = delta
            delta = nxt
        self.meas[:6] = m
        self.last = t
        K = self.P @ np.linalg.inv(self.P + self.R)
        self.x = self.xn + K @ (self.meas - self.xn)
        self.P = (np.eye(self.n) - K) @ self.P
        self.xn = self.F @ self.x
        self.P = self.F @ self.P @ self.F.T + self.Q
        for i in range(self.steps + 1):
            self.pred[i] = np.linalg.matrix_power(self.F, i) @ self.x

    def observe_time(self, t):
        if t <= self.last:
            return
        self.x = self.xn
        self.xn = self.F @ self.x
        self.P = self.F @ self.P @ self.F.T + self.Q

    def get(self, t):
        if t > self.last + self.horison:
            return np.zeros(6)
        u = (t - self.last) / self.dt
        lo = int(u)
        u -= lo
        lo = min(max(lo, 0), self.steps)
        hi = min(lo + 1, self.steps)
        return (1.0 - u) * self.pred[lo, :6] + u * self.pred[hi, :6]


def gen_kalman(order, seed, H=64):
    """An actor-like event stream (actor.cpp:155-197): a wrench observed every 5 ms, time ticks
    in between, and the H-step table an update at the same instant would sample."""
    rng = np.random.default_rng(seed)
    kf = KalmanForecastNp(order, 0.005, 0.3, np.zeros(6))
    events, tables = [], []
    for j in range(40):
        t = 0.005 * j
        w = np.array([20 + 5 * math.sin(4 * t), 3 * math.cos(2 * t), -1 + t, 0.1, -0.2, 0.05 * j]) + rng.normal(0, 0.2, 6)
        kf.observe(w, t)
        events.append(np.concatenate([[0.0, t], w]))
        for q in (0.001, 0.002, 0.003):
            kf.observe_time(t + q)
            events.append(np.concatenate([[1.0, t + q], np.zeros(6)]))
        if j % 8 == 7:
            tables.append(np.array([kf.get(t + 0.004 + 0.01 * k) for k in range(H)]))
            events.append(np.concatenate([[2.0, t + 0.004], np.zeros(6)]))
    return dict(order=np.array(order), time_step=np.array(0.005), horison=np.array(0.3),
                events=np.array(events), tables=np.array(tables), H=np.array(H), dt=np.array(0.01))


def huddled():
    x = np.zeros(31)
    x[:12] = [0.2, 0.2, math.pi / 4, 0.0, math.pi / 5, 0.0, -math.pi / 2, 0.0, 2, math.pi / 4, 0.025, 0.025]
    x[30] = 100.0
    return x


def gen_kinematics(rob, n=24, seed=1):
    rng = np.random.default_rng(seed)
    x0 = huddled()
    qs, vs, taus, outs = [], [], [], []
    for i in range(n):
        q = x0[:12] + rng.normal(0, 0.6, 12) * (1 if i else 0)
        q[10:] = np.abs(q[10:]) * 0.05 + 0.01
        v = rng.normal(0, 1.0, 12)
        tau = np.zeros(12)
        tau[3:10] = rng.normal(0, 5.0, 7)
        M = rob.mass_matrix(q)
        a = np.linalg.solve(M, tau)
        k = kin(rob, q, v)
        fd = fd_world_velocity(rob, q, v, EE_LINK)
        assert np.allclose(fd, k["vee"], atol=1e-6), (fd, k["vee"])
        qs.append(q); vs.append(v); taus.append(tau)
        outs.append(np.concatenate([a, k["ee"], k["am"], k["J"].reshape(-1), k["vee"], M.reshape(-1)]))
    return np.array(qs), np.array(vs), np.array(taus), np.array(outs)


def near_limits():
    """HUDDLED with joint 1 and joint 4 just inside TrackPoint's upper limits (2.8973, 0.0698)."""
    x = huddled()
    x[3], x[6] = 2.89, 0.06
    return x


def gen_updates(rob, S, K, H, updates, seed, smoothing=None, track_point=False, energy0=None):
    dt = 0.01
    x0 = near_limits() if track_point else huddled()
    objective = track_point_cost if track_point else None
    if energy0 is not None:   # energy_cost alone (every other term disabled), tank started at energy0
        x0[30] = energy0
        objective = energy_only_cost
    m = MPPI(rob, S, K, H, dt, VAR, CMIN, CMAX, x0, smoothing, objective=objective, energy=energy0 is not None)
    rng = np.random.default_rng(seed)
    sd = np.sqrt(VAR)
    forecast = np.zeros((H, 6))
    forecast[:, 0] = 20.0
    x = x0.copy()
    rec = {k: [] for k in ("eps", "costs", "weights", "gradient", "U", "opt_cost", "time")}
    for j in range(updates):
        t = 0.05 * j
        n = m.draws(t)
        eps = rng.standard_normal((n, 12)) * sd
        m.update(x, t, eps, forecast)
        rec["eps"].append(eps)
        rec["costs"].append(m.cost.copy())
        rec["weights"].append(m.w.copy())
        rec["gradient"].append(m.g.copy())
        rec["U"].append(m.U.copy())
        rec["opt_cost"].append(m.opt_cost)
        rec["time"].append(t)
        print("  update %d: min cost %.6e argmin %d" % (j, np.nanmin(m.cost), int(np.nanargmin(m.cost))))
    out = dict(S=S, K=K, H=H, x0=x0, forecast=forecast,
               eps=np.concatenate(rec["eps"]), eps_counts=np.array([len(e) for e in rec["eps"]]),
               costs=np.array(rec["costs"]), weights=np.array(rec["weights"]), gradient=np.array(rec["gradient"]),
               U=np.array(rec["U"]), opt_cost=np.array(rec["opt_cost"]), time=np.array(rec["time"]),
               smoothing=np.array(smoothing if smoothing else (0, 0)),
               objective=np.array("track_point" if track_point else ("energy_only" if energy0 is not None else "assisted_manipulation")),
               energy=np.array(1 if energy0 is not None else 0),
               track_point=TP_POINT)
    return out


def main():
    rob = Robot()
    if "--kalman" in sys.argv or not os.path.exists(os.path.join(HERE, "kalman.npz")):
        print("Kalman forecast fixtures (orders 1, 2)")
        k1, k2 = gen_kalman(1, 41), gen_kalman(2, 42)
        np.savez_compressed(os.path.join(HERE, "kalman.npz"), **{"o1_" + k: v for k, v in k1.items()},
                            **{"o2_" + k: v for k, v in k2.items()})
        if "--kalman" in sys.argv:
            return
    if "--energy" in sys.argv or not os.path.exists(os.path.join(HERE, "nle.npz")):
        print("NLE fixtures (complex-step Lagrangian)")
        rng = np.random.default_rng(5)
        nq, nv, nn = [], [], []
        for i in range(12):
            qq = huddled()[:12] + rng.normal(0, 0.6, 12) * (1 if i else 0)
            qq[10:] = np.abs(qq[10:]) * 0.05 + 0.01
            vv = rng.normal(0, 1.5, 12)
            nq.append(qq); nv.append(vv); nn.append(rob.nle(qq, vv))
        ru, rE, re0 = energy_rollouts(rob)
        np.savez_compressed(os.path.join(HERE, "nle.npz"), q=np.array(nq), v=np.array(nv), nle=np.array(nn),
                            roll_u=ru, roll_E=rE, roll_E0=re0)
        print("update fixtures: 16 x 8, energy tank enabled (E0 = 15)")
        np.savez_compressed(os.path.join(HERE, "update_s16_h8_energy.npz"),
                            **gen_updates(rob, 16, 4, 8, 4, seed=24, energy0=15.0))
        if "--energy" in sys.argv:
            return
    if "--ee" in sys.argv or not os.path.exists(os.path.join(HERE, "end_effector.npz")):
        print("end-effector orientation / acceleration fixtures (complex step)")
        q, v, tau, out = gen_end_effector(rob)
        np.savez_compressed(os.path.join(HERE, "end_effector.npz"), q=q, v=v, tau=tau, out=out)
        if "--ee" in sys.argv:
            return
    print("kinematics fixtures")
    q, v, tau, out = gen_kinematics(rob)
    np.savez_compressed(os.path.join(HERE, "kinematics.npz"), q=q, v=v, tau=tau, out=out)
    print("SG weights")
    np.savez_compressed(os.path.join(HERE, "sg_weights.npz"), w10_1=sg_weights(10, 1), w5_2=sg_weights(5, 2),
                        w3_3=sg_weights(3, 3))
    print("update fixtures: 16 x 8")
    np.savez_compressed(os.path.join(HERE, "update_s16_h8.npz"), **gen_updates(rob, 16, 4, 8, 4, seed=21))
    print("update fixtures: 24 x 16 with SG(4, 1)")
    np.savez_compressed(os.path.join(HERE, "update_s24_h16_sg.npz"), **gen_updates(rob, 24, 6, 16, 4, seed=22, smoothing=(4, 1)))
    print("update fixtures: 16 x 8, TrackPoint objective (all terms)")
    np.savez_compressed(os.path.join(HERE, "update_s16_h8_trackpoint.npz"),
                        **gen_updates(rob, 16, 4, 8, 4, seed=23, track_point=True))
    if "--config1" in sys.argv:
        print("update fixtures: config 1 (128 x 32)")
        np.savez_compressed(os.path.join(HERE, "update_s128_h32.npz"), **gen_updates(rob, 128, 20, 32, 3, seed=12345))


if __name__ == "__main__":
    main()
