"""Shim modules that let the reference's own ``drone_2d_env.py`` be imported in this
container, used ONLY by ``make_golden.py`` to record golden vectors.

Test infrastructure, never shipped and never imported by the product package.

Why shims exist: the reference imports ``pymunk`` (Chipmunk2D), ``pygame`` and ``gym``
(``drone_2d_env.py:1-10``, ``Drone.py:1-5``, ``obstacles.py:1-4``); none is installed and
there is no network.  ``pygame``/``gym`` are only used for rendering / the ``gym.Env`` base
class / ``spaces.Box``, so their shims are inert.  The ``pymunk`` shim carries ONE piece of
real behaviour: ``Space.step`` -- a plain-Python fp64 restatement of Chipmunk2D 7.0.x's
``cpSpaceStep`` for exactly the configuration the reference builds (3 dynamic bodies, 6
``PivotJoint`` with ``error_bias = 0``, sensor shapes, circle obstacles), per SURVEY.md
Appendix A.  Chipmunk's source is not in the container, so THE PHYSICS IN THESE VECTORS IS
PARITY-UNPINNED (it is this restatement, cross-checked against the independent C oracle and
physics known-answer tests).  Everything else recorded -- spawn logic, the QPMI2D path and
scipy ``fminbound`` closest-point search, k-nearest sensing, the 27-dim observation, the
reward terms, termination and ``info`` -- is executed by the reference's own unmodified
Python.

Chipmunk2D 7.0.x functions restated (third-party C, pymunk 6.x bundle, not vendored):
  cpSpaceStep (cpSpaceStep.c), cpBodyUpdatePosition / cpBodyUpdateVelocity /
  cpBodyApplyForceAtLocalPoint / cpBodyGetVelocityAtLocalPoint (cpBody.c),
  PivotJoint preStep / applyCachedImpulse / applyImpulse (cpPivotJoint.c),
  k_tensor / relative_velocity / apply_impulses (chipmunk_private.h, cpConstraint.h),
  cpMomentForPoly (chipmunk.c), cpBoxShapeNew2 vertex order (cpPolyShape.c),
  CircleToPoly contact test (cpCollision.c: contact iff dist(center, box) <= r).
"""
from __future__ import annotations

import math
import sys
import types
from typing import NamedTuple


# --------------------------------------------------------------------------- Vec2d
class Vec2d(NamedTuple):
    x: float
    y: float

    def __add__(self, o):  # type: ignore[override]
        return Vec2d(self.x + o[0], self.y + o[1])

    def __sub__(self, o):
        return Vec2d(self.x - o[0], self.y - o[1])

    def get_distance(self, o) -> float:
        # pymunk 6 Vec2d.get_distance: math.sqrt((x-ox)**2 + (y-oy)**2)
        return math.sqrt((self.x - o[0]) ** 2 + (self.y - o[1]) ** 2)


def _tvect(cos_a, sin_a, vx, vy):
    # cpTransformVect with transform (a=cos, b=sin, c=-sin, d=cos)
    return (cos_a * vx + (-sin_a) * vy, sin_a * vx + cos_a * vy)


def _tpoint(cos_a, sin_a, px, py, vx, vy):
    # cpTransformPoint; tx = p.x - (cog.x*cos - cog.y*sin) = p.x - 0.0 for cog = 0
    tx = px - (0.0 * cos_a - 0.0 * sin_a)
    ty = py - (0.0 * sin_a + 0.0 * cos_a)
    return (cos_a * vx + (-sin_a) * vy + tx, sin_a * vx + cos_a * vy + ty)


# --------------------------------------------------------------------------- Body
class Body:
    DYNAMIC = 0
    KINEMATIC = 1
    STATIC = 2

    def __init__(self, mass=0.0, moment=0.0, body_type=DYNAMIC):
        self.body_type = body_type
        self.m = float(mass)
        self.i = float(moment)
        self.m_inv = math.inf if self.m == 0.0 else 1.0 / self.m
        self.i_inv = math.inf if self.i == 0.0 else 1.0 / self.i
        self.px = 0.0
        self.py = 0.0
        self.a = 0.0
        self.cos_a = 1.0
        self.sin_a = 0.0
        self.vx = 0.0
        self.vy = 0.0
        self.w = 0.0
        self.fx = 0.0
        self.fy = 0.0
        self.t = 0.0

    # cpBodySetPosition / cpBodyGetPosition (cog = 0 -> exact round trip)
    @property
    def position(self):
        return Vec2d(self.px, self.py)

    @position.setter
    def position(self, p):
        self.px = float(p[0])
        self.py = float(p[1])

    @property
    def angle(self):
        return self.a

    @angle.setter
    def angle(self, a):
        self.a = float(a)
        self.cos_a = math.cos(self.a)
        self.sin_a = math.sin(self.a)

    @property
    def velocity(self):
        return Vec2d(self.vx, self.vy)

    @property
    def angular_velocity(self):
        return self.w

    def apply_force_at_local_point(self, force, point=(0, 0)):
        # cpBodyApplyForceAtLocalPoint -> cpBodyApplyForceAtWorldPoint
        fwx, fwy = _tvect(self.cos_a, self.sin_a, float(force[0]), float(force[1]))
        wpx, wpy = _tpoint(self.cos_a, self.sin_a, self.px, self.py, float(point[0]), float(point[1]))
        cgx, cgy = _tpoint(self.cos_a, self.sin_a, self.px, self.py, 0.0, 0.0)
        self.fx = self.fx + fwx
        self.fy = self.fy + fwy
        rx = wpx - cgx
        ry = wpy - cgy
        self.t += rx * fwy - ry * fwx

    def apply_force_at_world_point(self, force, point):  # initial_movement only (never called)
        self.fx += float(force[0])
        self.fy += float(force[1])
        rx = float(point[0]) - self.px
        ry = float(point[1]) - self.py
        self.t += rx * float(force[1]) - ry * float(force[0])

    def velocity_at_local_point(self, point):
        # cpBodyGetVelocityAtLocalPoint: v + perp(r) * w with r = T.vect(point - cog)
        rx, ry = _tvect(self.cos_a, self.sin_a, float(point[0]), float(point[1]))
        return Vec2d(self.vx + (-ry) * self.w, self.vy + rx * self.w)

    # cpBodyUpdatePosition (v_bias = w_bias = 0)
    def _update_position(self, dt):
        self.px = self.px + (self.vx + 0.0) * dt
        self.py = self.py + (self.vy + 0.0) * dt
        self.angle = self.a + (self.w + 0.0) * dt

    # cpBodyUpdateVelocity
    def _update_velocity(self, gx, gy, damping, dt):
        self.vx = self.vx * damping + (gx + self.fx * self.m_inv) * dt
        self.vy = self.vy * damping + (gy + self.fy * self.m_inv) * dt
        self.w = self.w * damping + self.t * self.i_inv * dt
        self.fx = self.fy = 0.0
        self.t = 0.0


# --------------------------------------------------------------------------- shapes
class Shape:
    def __init__(self, body):
        self.body = body
        self.sensor = False
        self.collision_type = 0
        self.color = None
        self.elasticity = 0.0
        self.friction = 0.0


class Poly(Shape):
    def __init__(self, body, vertices):
        super().__init__(body)
        self._verts = [Vec2d(float(v[0]), float(v[1])) for v in vertices]

    @staticmethod
    def create_box(body, size=(10, 10), radius=0):
        hw = size[0] / 2.0
        hh = size[1] / 2.0
        # cpBoxShapeNew2: (r,b), (r,t), (l,t), (l,b)
        return Poly(body, [(hw, -hh), (hw, hh), (-hw, hh), (-hw, -hh)])

    def get_vertices(self):
        return list(self._verts)


class Circle(Shape):
    def __init__(self, body, radius, offset=(0, 0)):
        super().__init__(body)
        self.radius = float(radius)


class Segment(Shape):
    pass


def moment_for_poly(mass, vertices, offset=(0, 0), radius=0):
    # cpMomentForPoly
    n = len(vertices)
    s1 = 0.0
    s2 = 0.0
    for i in range(n):
        v1x = float(vertices[i][0]) + offset[0]
        v1y = float(vertices[i][1]) + offset[1]
        v2x = float(vertices[(i + 1) % n][0]) + offset[0]
        v2y = float(vertices[(i + 1) % n][1]) + offset[1]
        a = v2x * v1y - v2y * v1x
        b = (v1x * v1x + v1y * v1y) + (v1x * v2x + v1y * v2y) + (v2x * v2x + v2y * v2y)
        s1 += a * b
        s2 += a
    return (mass * s1) / (6.0 * s2)


# --------------------------------------------------------------------------- joints
class PivotJoint:
    def __init__(self, a, b, anchor_a, anchor_b):
        self.a = a
        self.b = b
        self.anchor_a = (float(anchor_a[0]), float(anchor_a[1]))
        self.anchor_b = (float(anchor_b[0]), float(anchor_b[1]))
        self.error_bias = (1.0 - 0.1) ** 60.0  # Chipmunk default, overwritten to 0 by Drone.py
        self.max_bias = math.inf
        self.max_force = math.inf
        self.jAcc = [0.0, 0.0]

    def _pre_step(self, dt):
        a, b = self.a, self.b
        self.r1 = _tvect(a.cos_a, a.sin_a, self.anchor_a[0] - 0.0, self.anchor_a[1] - 0.0)
        self.r2 = _tvect(b.cos_a, b.sin_a, self.anchor_b[0] - 0.0, self.anchor_b[1] - 0.0)
        r1x, r1y = self.r1
        r2x, r2y = self.r2
        # k_tensor
        m_sum = a.m_inv + b.m_inv
        k11, k12, k21, k22 = m_sum, 0.0, 0.0, m_sum
        r1xsq = r1x * r1x * a.i_inv
        r1ysq = r1y * r1y * a.i_inv
        r1nxy = -r1x * r1y * a.i_inv
        k11 += r1ysq
        k12 += r1nxy
        k21 += r1nxy
        k22 += r1xsq
        r2xsq = r2x * r2x * b.i_inv
        r2ysq = r2y * r2y * b.i_inv
        r2nxy = -r2x * r2y * b.i_inv
        k11 += r2ysq
        k12 += r2nxy
        k21 += r2nxy
        k22 += r2xsq
        det = k11 * k22 - k12 * k21
        det_inv = 1.0 / det
        self.k = (k22 * det_inv, -k12 * det_inv, -k21 * det_inv, k11 * det_inv)
        # bias = clamp(delta * -bias_coef/dt, max_bias); bias_coef = 1 - error_bias^dt
        dx = (b.px + r2x) - (a.px + r1x)
        dy = (b.py + r2y) - (a.py + r1y)
        coef = -(1.0 - self.error_bias ** dt) / dt
        self.bias = (dx * coef, dy * coef)

    @staticmethod
    def _apply(body, jx, jy, rx, ry):
        body.vx = body.vx + jx * body.m_inv
        body.vy = body.vy + jy * body.m_inv
        body.w += body.i_inv * (rx * jy - ry * jx)

    def _apply_impulses(self, jx, jy):
        self._apply(self.a, -jx, -jy, self.r1[0], self.r1[1])
        self._apply(self.b, jx, jy, self.r2[0], self.r2[1])

    def _apply_cached(self, dt_coef):
        self._apply_impulses(self.jAcc[0] * dt_coef, self.jAcc[1] * dt_coef)

    def _apply_impulse(self):
        a, b = self.a, self.b
        r1x, r1y = self.r1
        r2x, r2y = self.r2
        v1x = a.vx + (-r1y) * a.w
        v1y = a.vy + r1x * a.w
        v2x = b.vx + (-r2y) * b.w
        v2y = b.vy + r2x * b.w
        vrx = v2x - v1x
        vry = v2y - v1y
        ux = self.bias[0] - vrx
        uy = self.bias[1] - vry
        ka, kb, kc, kd = self.k
        jx = ux * ka + uy * kb
        jy = ux * kc + uy * kd
        ox, oy = self.jAcc
        self.jAcc = [ox + jx, oy + jy]  # clamp to max_force*dt = inf is a no-op
        self._apply_impulses(self.jAcc[0] - ox, self.jAcc[1] - oy)


# --------------------------------------------------------------------------- space
class _Handler:
    def __init__(self):
        self.begin = None


class Space:
    def __init__(self):
        self.gravity = Vec2d(0.0, 0.0)
        self.damping = 1.0
        self.iterations = 10
        self.curr_dt = 0.0
        self._bodies = []
        self._shapes = []
        self._constraints = []
        self._handlers = {}

    @property
    def bodies(self):
        return list(self._bodies)

    def add(self, *objs):
        for o in objs:
            if isinstance(o, Body):
                self._bodies.append(o)
            elif isinstance(o, Shape):
                self._shapes.append(o)
            elif isinstance(o, PivotJoint):
                self._constraints.append(o)

    def add_collision_handler(self, ta, tb):
        h = self._handlers.setdefault((ta, tb), _Handler())
        return h

    @staticmethod
    def _box_circle_touch(poly: Poly, circ: Circle) -> bool:
        b = poly.body
        hx = max(abs(v.x) for v in poly._verts)
        hy = max(abs(v.y) for v in poly._verts)
        cx, cy = circ.body.px, circ.body.py
        dx = cx - b.px
        dy = cy - b.py
        lx = dx * b.cos_a + dy * b.sin_a
        ly = -dx * b.sin_a + dy * b.cos_a
        qx = min(max(lx, -hx), hx)
        qy = min(max(ly, -hy), hy)
        ex = lx - qx
        ey = ly - qy
        return ex * ex + ey * ey <= circ.radius * circ.radius

    def step(self, dt):
        dt = float(dt)
        prev_dt = self.curr_dt
        self.curr_dt = dt
        dyn = [b for b in self._bodies if b.body_type == Body.DYNAMIC]
        for b in dyn:
            b._update_position(dt)
        # collision detection + begin callbacks (only the (1,2) handler exists)
        for (ta, tb), h in self._handlers.items():
            if h.begin is None:
                continue
            polys = [s for s in self._shapes if isinstance(s, Poly) and s.collision_type == ta]
            circs = [s for s in self._shapes if isinstance(s, Circle) and s.collision_type == tb]
            for p in polys:
                for c in circs:
                    if self._box_circle_touch(p, c):
                        h.begin(None, self, None)
        for c in self._constraints:
            c._pre_step(dt)
        damping = self.damping ** dt
        for b in dyn:
            b._update_velocity(float(self.gravity[0]), float(self.gravity[1]), damping, dt)
        dt_coef = 0.0 if prev_dt == 0.0 else dt / prev_dt
        for c in self._constraints:
            c._apply_cached(dt_coef)
        for _ in range(self.iterations):
            for c in self._constraints:
                c._apply_impulse()

    def debug_draw(self, *_a, **_k):
        pass


# --------------------------------------------------------------------------- install
def install() -> None:
    """Register the shim modules in ``sys.modules`` (pymunk, pygame, gym)."""
    pm = types.ModuleType("pymunk")
    for name, obj in dict(Vec2d=Vec2d, Body=Body, Poly=Poly, Circle=Circle, Segment=Segment,
                          Shape=Shape, PivotJoint=PivotJoint, Space=Space,
                          moment_for_poly=moment_for_poly).items():
        setattr(pm, name, obj)
    shapes = types.ModuleType("pymunk.shapes")
    shapes.Circle = Circle
    shapes.Poly = Poly
    pm.shapes = shapes
    pgu = types.ModuleType("pymunk.pygame_util")
    pgu.positive_y_is_up = True
    pgu.DrawOptions = lambda *a, **k: types.SimpleNamespace(flags=0)
    pm.pygame_util = pgu
    pm.SpaceDebugDrawOptions = types.SimpleNamespace(DRAW_SHAPES=1)
    sys.modules["pymunk"] = pm
    sys.modules["pymunk.shapes"] = shapes
    sys.modules["pymunk.pygame_util"] = pgu

    pg = types.ModuleType("pygame")
    pg.Color = lambda *a, **k: a
    pg.init = lambda *a, **k: None
    pg.quit = lambda *a, **k: None
    pg.MOUSEBUTTONUP = 6
    pg.event = types.SimpleNamespace(get=lambda: [])
    pgl = types.ModuleType("pygame.locals")
    pgl.QUIT, pgl.KEYDOWN, pgl.K_ESCAPE = 12, 2, 27
    pg.locals = pgl
    sys.modules["pygame"] = pg
    sys.modules["pygame.locals"] = pgl

    gym = types.ModuleType("gym")

    class Env:  # gym.Env base: no behaviour used by the reference
        pass

    class Box:
        def __init__(self, low, high, shape=None, dtype=None):
            self.low, self.high, self.dtype = low, high, dtype
            self.shape = low.shape if shape is None else shape

    spaces = types.ModuleType("gym.spaces")
    spaces.Box = Box
    utils = types.ModuleType("gym.utils")
    utils.seeding = types.SimpleNamespace()
    gym.Env = Env
    gym.spaces = spaces
    gym.utils = utils
    sys.modules["gym"] = gym
    sys.modules["gym.spaces"] = spaces
    sys.modules["gym.utils"] = utils
