#!/usr/bin/env python3
"""Generate include/mppi_amd_frankaridgeback.h from the reference's robot.urdf.

Run in the build container (the reference is not present on the GPU box); the generated
header is committed.  It restates what Pinocchio v2.7.1's URDF parser builds from
src/frankaridgeback/model/robot.urdf (pinocchio_dynamics.cpp:53 `buildModelFromXML`):

  * urdfdom orders a link's children by joint name (std::map in ModelInterface::initTree),
    Pinocchio visits them depth first — this fixes the DoF order x, y, pivot, j1..j7, f1, f2
    (frankaridgeback/dof.hpp, state.hpp:112-114);
  * a fixed joint adds a frame at parent_frame.placement * origin and appends the child link's
    inertia to the parent *moving* joint (InertiaTpl::operator+= merge formula), skipping links
    whose inertia is exactly zero;
  * an origin rpy becomes urdfdom's quaternion (Rotation::setFromRPY + normalize), then
    Eigen's Quaternion::toRotationMatrix — the URDF's literal decimals are used (no M_PI);
  * an inertial origin rotates the inertia tensor: I_link = R I R^T about the com.

SURVEY.md Appendix A/B lists the result; tests/golden/gen_golden.py checks it against an
independent, unmerged numpy model.
"""
import math
import os
import sys
import xml.etree.ElementTree as ET

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
URDF = "/root/reference/src/frankaridgeback/model/robot.urdf"
OUT = os.path.join(REPO, "include", "mppi_amd_frankaridgeback.h")


# --- urdfdom / Eigen rotation conventions ---------------------------------------------------
def quat_from_rpy(roll, pitch, yaw):
    """urdf::Rotation::setFromRPY followed by normalize()."""
    phi, the, psi = roll / 2.0, pitch / 2.0, yaw / 2.0
    x = math.sin(phi) * math.cos(the) * math.cos(psi) - math.cos(phi) * math.sin(the) * math.sin(psi)
    y = math.cos(phi) * math.sin(the) * math.cos(psi) + math.sin(phi) * math.cos(the) * math.sin(psi)
    z = math.cos(phi) * math.cos(the) * math.sin(psi) - math.sin(phi) * math.sin(the) * math.cos(psi)
    w = math.cos(phi) * math.cos(the) * math.cos(psi) + math.sin(phi) * math.sin(the) * math.sin(psi)
    s = math.sqrt(x * x + y * y + z * z + w * w)
    if s == 0.0:
        return (0.0, 0.0, 0.0, 1.0)
    return (x / s, y / s, z / s, w / s)


def quat_matrix(q):
    """Eigen::Quaternion::toRotationMatrix (row-major 3x3 list)."""
    x, y, z, w = q
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return [
        [1.0 - (tyy + tzz), txy - twz, txz + twy],
        [txy + twz, 1.0 - (txx + tzz), tyz - twx],
        [txz - twy, tyz + twx, 1.0 - (txx + tyy)],
    ]


def matmul(a, b):
    return [[(a[i][0] * b[0][j] + a[i][1] * b[1][j]) + a[i][2] * b[2][j]
             for j in range(3)] for i in range(3)]


def matvec(a, v):
    return [(a[i][0] * v[0] + a[i][1] * v[1]) + a[i][2] * v[2] for i in range(3)]


def transpose(a):
    return [[a[j][i] for j in range(3)] for i in range(3)]


class SE3:
    def __init__(self, R=None, p=None):
        self.R = R if R is not None else [[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]]
        self.p = p if p is not None else [0.0, 0.0, 0.0]

    def __mul__(self, o):  # pinocchio SE3::operator*
        Rp = matvec(self.R, o.p)
        return SE3(matmul(self.R, o.R), [self.p[i] + Rp[i] for i in range(3)])


def parse_origin(el):
    o = el.find("origin")
    if o is None:
        return SE3()
    xyz = [float(v) for v in o.get("xyz", "0 0 0").split()]
    rpy = [float(v) for v in o.get("rpy", "0 0 0").split()]
    return SE3(quat_matrix(quat_from_rpy(*rpy)), xyz)


# --- Pinocchio InertiaTpl -----------------------------------------------------------------
class Inertia:
    """mass, lever (com), rotational inertia about com as full symmetric 3x3."""

    def __init__(self, m=0.0, c=None, I=None):
        self.m = m
        self.c = c if c is not None else [0.0, 0.0, 0.0]
        self.I = I if I is not None else [[0.0] * 3 for _ in range(3)]

    def is_zero(self):
        return self.m == 0.0 and all(v == 0.0 for v in self.c) and all(
            v == 0.0 for row in self.I for v in row)

    def se3_action(self, M):  # SE3::act(Inertia)
        Rc = matvec(M.R, self.c)
        c = [M.p[i] + Rc[i] for i in range(3)]
        I = matmul(matmul(M.R, self.I), transpose(M.R))
        return Inertia(self.m, c, I)

    def iadd(self, Yb):  # InertiaTpl::operator+=
        eps = 2.220446049250313e-16
        mab = self.m + Yb.m
        mab_inv = 1.0 / max(self.m + Yb.m, eps)
        AB = [self.c[i] - Yb.c[i] for i in range(3)]
        self.c = [self.c[i] * (self.m * mab_inv) for i in range(3)]
        self.c = [self.c[i] + (Yb.m * mab_inv) * Yb.c[i] for i in range(3)]
        mu = self.m * Yb.m * mab_inv
        # SkewSquare(AB) = [AB]x^2 = AB AB^T - |AB|^2 E
        n2 = AB[0] * AB[0] + AB[1] * AB[1] + AB[2] * AB[2]
        for i in range(3):
            for j in range(3):
                ss = AB[i] * AB[j] - (n2 if i == j else 0.0)
                self.I[i][j] = (self.I[i][j] + Yb.I[i][j]) - mu * ss
        self.m = mab


def link_inertia(link):
    inert = link.find("inertial")
    if inert is None:
        return Inertia()
    m = float(inert.find("mass").get("value"))
    o = parse_origin(inert)
    i = inert.find("inertia")
    g = lambda k: float(i.get(k, "0"))
    Iraw = [[g("ixx"), g("ixy"), g("ixz")], [g("ixy"), g("iyy"), g("iyz")], [g("ixz"), g("iyz"), g("izz")]]
    I = matmul(matmul(o.R, Iraw), transpose(o.R))
    return Inertia(m, list(o.p), I)


def build(urdf_path=URDF):
    root = ET.parse(urdf_path).getroot()
    links = {l.get("name"): l for l in root.findall("link")}
    joints = {j.get("name"): j for j in root.findall("joint")}  # top-level only
    children = {}
    child_links = set()
    for jname in sorted(joints):  # std::map order
        j = joints[jname]
        p = j.find("parent").get("link")
        c = j.find("child").get("link")
        children.setdefault(p, []).append(jname)
        child_links.add(c)
    roots = [l for l in links if l not in child_links]
    assert len(roots) == 1, roots
    bodies = []  # dicts
    frames = {}  # name -> (joint index, SE3 placement in joint frame)
    body_frame = {roots[0]: (-1, SE3())}

    def visit(link_name):
        for jname in children.get(link_name, []):
            j = joints[jname]
            child = j.find("child").get("link")
            parent_joint, parent_place = body_frame[link_name]
            origin = parse_origin(j)
            jtype = j.get("type")
            Y = link_inertia(links[child])
            if jtype == "fixed":
                place = parent_place * origin
                frames[jname] = (parent_joint, place)
                if parent_joint >= 0 and not Y.is_zero():
                    bodies[parent_joint]["Y"].iadd(Y.se3_action(place))
                body_frame[child] = (parent_joint, place)
            elif jtype in ("revolute", "prismatic", "continuous"):
                assert jtype != "continuous"
                axis = [float(v) for v in j.find("axis").get("xyz").split()]
                placement = parent_place * origin
                idx = len(bodies)
                Yj = Inertia()
                if not Y.is_zero():
                    Yj.iadd(Y.se3_action(SE3()))
                bodies.append(dict(name=jname, parent=parent_joint, type=jtype, axis=axis,
                                   placement=placement, Y=Yj))
                frames[jname] = (idx, SE3())
                body_frame[child] = (idx, SE3())
            else:
                raise ValueError(jtype)
            visit(child)

    visit(roots[0])
    return bodies, frames


def fmt(v):
    return repr(float(v))


def emit(bodies, frames):
    lines = []
    w = lines.append
    w("/* GENERATED by tools/gen_model.py from the reference's src/frankaridgeback/model/robot.urdf.")
    w(" * Do not edit.  Pinocchio v2.7.1 URDF-parser conventions (see the generator's docstring). */")
    w("#ifndef MPPI_AMD_FRANKARIDGEBACK_H")
    w("#define MPPI_AMD_FRANKARIDGEBACK_H")
    w("")
    w("#include <string.h>")
    w("#include \"mppi_amd.h\"")
    w("")
    w("/* body order = DoF order (frankaridgeback/dof.hpp): " + ", ".join(b["name"] for b in bodies) + " */")
    w("static inline void mppi_frankaridgeback_model(mppi_frankaridgeback_desc *d)")
    w("{")
    w("    memset(d, 0, sizeof(*d));")
    w("    d->nbodies = %d;" % len(bodies))
    for i, b in enumerate(bodies):
        w("    /* %d: %s (%s) */" % (i, b["name"], b["type"]))
        w("    d->bodies[%d].parent = %d;" % (i, b["parent"]))
        w("    d->bodies[%d].type = %s;" % (i, "MPPI_JOINT_REVOLUTE" if b["type"] == "revolute" else "MPPI_JOINT_PRISMATIC"))
        for k in range(3):
            w("    d->bodies[%d].axis[%d] = %s;" % (i, k, fmt(b["axis"][k])))
        for r in range(3):
            for c in range(3):
                w("    d->bodies[%d].rotation[%d] = %s;" % (i, 3 * r + c, fmt(b["placement"].R[r][c])))
        for k in range(3):
            w("    d->bodies[%d].translation[%d] = %s;" % (i, k, fmt(b["placement"].p[k])))
        Y = b["Y"]
        w("    d->bodies[%d].mass = %s;" % (i, fmt(Y.m)))
        for k in range(3):
            w("    d->bodies[%d].lever[%d] = %s;" % (i, k, fmt(Y.c[k])))
        sym = [Y.I[0][0], Y.I[0][1], Y.I[1][1], Y.I[0][2], Y.I[1][2], Y.I[2][2]]
        for k in range(6):
            w("    d->bodies[%d].inertia[%d] = %s;" % (i, k, fmt(sym[k])))
    for field, name in (("end_effector", "panda_grasp_joint"), ("arm_mount", "arm_mount_joint")):
        j, M = frames[name]
        w("    /* frame %s */" % name)
        w("    d->%s.parent = %d;" % (field, j))
        for r in range(3):
            for c in range(3):
                w("    d->%s.rotation[%d] = %s;" % (field, 3 * r + c, fmt(M.R[r][c])))
        for k in range(3):
            w("    d->%s.translation[%d] = %s;" % (field, k, fmt(M.p[k])))
    w("    d->gravity[0] = 0.0;")
    w("    d->gravity[1] = 0.0;")
    w("    d->gravity[2] = -9.81;")
    w("}")
    w("")
    w(DEFAULTS)
    w("#endif /* MPPI_AMD_FRANKARIDGEBACK_H */")
    return "\n".join(lines) + "\n"


DEFAULTS = r'''
static inline mppi_barrier mppi_barrier_make(double bound, double scale)
{
    mppi_barrier b;
    b.bound = bound;
    b.scale = scale;
    b.maximum_cost = 1e10;  /* cost.hpp:57, :88 default */
    return b;
}

static inline mppi_quadratic mppi_quadratic_make(double c, double l, double q)
{
    mppi_quadratic r;
    r.constant_cost = c;
    r.linear_cost = l;
    r.quadratic_cost = q;
    return r;
}

/* AssistedManipulation::DEFAULT_CONFIGURATION (assisted_manipulation.hpp:133-206). */
static inline void mppi_assisted_manipulation_default(mppi_assisted_manipulation_desc *a)
{
    static const double lower[12][2] = {{-2.0, 0.0}, {-2.0, 0.0}, {-6.28, 0.0}, {-2.8, 10.0},
        {-1.745, 10.0}, {-2.8, 10.0}, {-3.0718, 10.0}, {-2.7925, 10.0}, {0.349, 10.0},
        {-2.967, 10.0}, {0.0, 0.0}, {0.0, 0.0}};
    static const double upper[12][2] = {{2.0, 0.0}, {2.0, 0.0}, {6.28, 0.0}, {2.8, 10.0},
        {1.745, 10.0}, {2.8, 10.0}, {0.0, 10.0}, {2.7925, 10.0}, {4.53785, 10.0},
        {2.967, 10.0}, {0.5, 0.0}, {0.5, 0.0}};
    static const double velocity[12] = {1000.0, 1000.0, 100.0, 0.5, 1.0, 2.0, 3.0, 4.0, 5.0,
        6.0, 0.0, 0.0};
    static const double radii[8] = {0.75, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1};
    int i;
    memset(a, 0, sizeof(*a));
    a->enable_joint_limit = 1;
    a->enable_self_collision_limit = 1;
    a->enable_workspace_limit = 1;
    a->enable_energy_limit = 0;
    a->enable_velocity_cost = 1;
    a->enable_trajectory_cost = 1;
    a->enable_manipulability_cost = 1;
    for (i = 0; i < 12; i++) {
        a->lower_joint_limit[i] = mppi_barrier_make(lower[i][0], lower[i][1]);
        a->upper_joint_limit[i] = mppi_barrier_make(upper[i][0], upper[i][1]);
        a->velocity_cost[i] = mppi_quadratic_make(0.0, 0.0, velocity[i]);
    }
    a->self_collision_limit = mppi_barrier_make(0.0, 1.0);
    for (i = 0; i < 8; i++)
        a->self_collision_radii[i] = radii[i];
    a->workspace_limit_above = mppi_barrier_make(0.0, 1.0);
    a->workspace_limit_infront = mppi_barrier_make(0.0, 1.0);
    a->workspace_limit_reach = mppi_barrier_make(1.0, 1.0);
    a->workspace_cost_yaw = mppi_quadratic_make(0.0, 0.0, 400.0);
    a->energy_limit_below = mppi_barrier_make(0.0, 10.0);
    a->energy_limit_above = mppi_barrier_make(20.0, 10.0);
    a->trajectory_target_scale = 1e-2;
    a->trajectory_target_maximum = 1.0;
    a->trajectory_position_cost = mppi_quadratic_make(100.0, 0.0, 500.0);
    a->trajectory_position_threshold = 0.0;
    a->trajectory_velocity_cost = mppi_quadratic_make(0.0, 0.0, 500.0);
    a->trajectory_velocity_minimum = 0.1;
    a->trajectory_velocity_maximum = 5.0;
    a->trajectory_velocity_dropoff = 2.0;
    a->manipulability_cost = mppi_quadratic_make(0.0, 0.0, 10.0);
    a->has_forecast = 1;
}

/* TrackPoint::DEFAULT_CONFIGURATION (frankaridgeback/objective/track_point.hpp:72-107). */
static inline void mppi_track_point_default(mppi_track_point_desc *t)
{
    static const double lower[12][2] = {{-2.0, 1.0}, {-2.0, 0.0}, {-6.28, 0.0}, {-2.8, 10.0},
        {-1.745, 50.0}, {-2.8, 10.0}, {-3.0718, 10.0}, {-2.7925, 10.0}, {0.349, 10.0},
        {-2.967, 10.0}, {0.0, 10.0}, {0.0, 10.0}};
    static const double upper[12][2] = {{2.0, 0.0}, {2.0, 0.0}, {6.28, 0.0}, {2.8, 10.0},
        {1.745, 50.0}, {2.8, 10.0}, {0.0, 10.0}, {2.7925, 10.0}, {4.53785, 10.0},
        {2.967, 10.0}, {0.5, 10.0}, {0.5, 10.0}};
    static const double radii[8] = {0.75, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1};
    int i;
    memset(t, 0, sizeof(*t));
    t->point[0] = 1.0;
    t->point[1] = 1.0;
    t->point[2] = 1.0;
    t->enable_joint_limits = 1;
    t->enable_self_collision_avoidance = 0;
    t->enable_power_limit = 0;
    t->enable_reach_limits = 0;
    for (i = 0; i < 12; i++) {
        t->lower_joint_limit[i] = mppi_barrier_make(lower[i][0], lower[i][1]);
        t->upper_joint_limit[i] = mppi_barrier_make(upper[i][0], upper[i][1]);
    }
    t->self_collision_limit = mppi_barrier_make(0.0, 1.0);
    for (i = 0; i < 8; i++)
        t->self_collision_radii[i] = radii[i];
    t->maximum_reach_limit = mppi_barrier_make(0.8, 1.0);
}

/* make_state(Preset::HUDDLED) (frankaridgeback/state.cpp:15-18): energy 100. */
static inline void mppi_frankaridgeback_huddled(double x[MPPI_FR_STATE])
{
    static const double pi = 3.14159265358979323846;
    static const double q[12] = {0.2, 0.2, pi / 4, 0.0, pi / 5, 0.0, -pi / 2, 0.0, 2, pi / 4,
        0.025, 0.025};
    int i;
    for (i = 0; i < MPPI_FR_STATE; i++)
        x[i] = 0.0;
    for (i = 0; i < 12; i++)
        x[i] = q[i];
    x[30] = 100.0;
}

/* The mppi::Configuration numbers of BaseTest::DEFAULT_CONFIGURATION (test/case/base.hpp:69-101). */
static const double MPPI_FR_DEFAULT_VARIANCE[12] = {0.1, 0.1, 0.2, 7.5, 7.5, 7.5, 7.5, 7.5, 7.5,
    7.5, 0.0, 0.0};
static const double MPPI_FR_DEFAULT_CONTROL_MIN[12] = {-0.5, -0.5, -1.0, -100.0, -100.0, -100.0,
    -100.0, -100.0, -100.0, -100.0, -0.05, -0.05};
static const double MPPI_FR_DEFAULT_CONTROL_MAX[12] = {0.5, 0.5, 1.0, 100.0, 100.0, 100.0,
    100.0, 100.0, 100.0, 100.0, 0.05, 0.05};
'''


def main():
    bodies, frames = build()
    text = emit(bodies, frames)
    with open(OUT, "w") as f:
        f.write(text)
    print("wrote", OUT, "bodies:", [b["name"] for b in bodies])
    for b in bodies:
        print(b["name"], b["parent"], b["type"], b["axis"], "m=%.6f" % b["Y"].m, b["placement"].p)
    for n in ("panda_grasp_joint", "arm_mount_joint"):
        print(n, frames[n][0], frames[n][1].p)


if __name__ == "__main__":
    sys.exit(main())
