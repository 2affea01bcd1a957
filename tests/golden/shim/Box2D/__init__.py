"""TEST-ONLY stand-in for PyBox2D 2.3.10 (absent from this image).

Implements exactly the pybox2d surface the reference calls (SURVEY.md 8(b),
row "L0 surface"), with float32 arithmetic for every b2Vec2 / b2Mat22 op and
with ALL geometry and physics delegated to the C oracle
(oracle/build/libmas_oracle.so): b2PolygonShape::Set/SetAsBox, TestPoint,
RayCast, and b2World::Step (ora_world_step).  Running the reference's own
simulation.py / semantics.py / masurvival_env.py over this shim pins the
oracle's rules / observation / reward restatement to the reference code;
physics itself stays the oracle's (Box2D parity is unpinned).

Canonical orders (where Box2D's depend on its dynamic tree / contact lists):
the golden generator registers the env's groups in dict order in
``CANONICAL_GROUPS``; ray casts and AABB queries report fixtures in that group
order, bodies in group list order.  Physics statics: walls group, then boxes.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, byref, c_float, c_int32

import numpy as np

f32 = np.float32

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.abspath(os.path.join(_HERE, '..', '..', '..', '..', 'oracle', 'build', 'libmas_oracle.so'))
_L = ctypes.CDLL(_LIB_PATH)

MAX_DYN, MAX_STAT = 16, 72


class _V2(Structure):
    _fields_ = [('x', c_float), ('y', c_float)]


class _Rot(Structure):
    _fields_ = [('s', c_float), ('c', c_float)]


class _Poly(Structure):
    _fields_ = [('count', c_int32), ('v', _V2 * 8), ('n', _V2 * 8)]


class _Cmem(Structure):
    _fields_ = [('touching', c_int32), ('ni', c_float), ('ti', c_float)]


class _World(Structure):
    _fields_ = [
        ('n_dyn', c_int32), ('active', c_int32 * MAX_DYN), ('c', _V2 * MAX_DYN), ('a', c_float * MAX_DYN),
        ('v', _V2 * MAX_DYN), ('w', c_float * MAX_DYN), ('sleep_time', c_float * MAX_DYN),
        ('awake', c_int32 * MAX_DYN), ('radius', c_float), ('inv_mass', c_float), ('inv_I', c_float),
        ('lin_damp', c_float), ('ang_damp', c_float), ('n_stat', c_int32), ('sp', _V2 * MAX_STAT),
        ('sa', c_float * MAX_STAT), ('sq', _Rot * MAX_STAT), ('spoly', _Poly * MAX_STAT),
        ('aa', (_Cmem * MAX_DYN) * MAX_DYN), ('as_', (_Cmem * MAX_STAT) * MAX_DYN), ('inv_dt0', c_float),
    ]


_L.ora_world_sizeof.restype = c_int32
assert _L.ora_world_sizeof() == ctypes.sizeof(_World), 'ora_world layout mismatch'
_L.ora_sincos.argtypes = [c_float, POINTER(c_float), POINTER(c_float)]
_L.ora_poly_set_as_box.argtypes = [POINTER(_Poly), c_float, c_float]
_L.ora_poly_set.argtypes = [POINTER(_Poly), POINTER(_V2), c_int32]
_L.ora_poly_test_point.restype = c_int32
_L.ora_poly_test_point.argtypes = [POINTER(_Poly), _V2, _Rot, _V2]
_L.ora_circle_test_point.restype = c_int32
_L.ora_circle_test_point.argtypes = [c_float, _V2, _V2]
_L.ora_ray_circle.restype = c_int32
_L.ora_ray_circle.argtypes = [c_float, _V2, _V2, _V2, c_float, POINTER(c_float)]
_L.ora_ray_poly.restype = c_int32
_L.ora_ray_poly.argtypes = [POINTER(_Poly), _V2, _Rot, _V2, _V2, c_float, POINTER(c_float)]
_L.ora_body_mass.argtypes = [c_float, c_float, POINTER(c_float), POINTER(c_float)]
_L.ora_world_step.argtypes = [POINTER(_World), c_float, c_int32, c_int32]

# group registry: filled by the golden generator after env construction
CANONICAL_GROUPS = []   # groups in Simulation.groups dict order
STATIC_GROUPS = []      # physics static order: [walls group, boxes group]


def _sincos(angle):
    s, c = c_float(), c_float()
    _L.ora_sincos(c_float(f32(angle)), byref(s), byref(c))
    return f32(s.value), f32(c.value)


class b2Vec2:
    __slots__ = ('x', 'y')
    __array_ufunc__ = None  # numpy scalars defer to __rmul__ / __radd__

    def __init__(self, *args, **kw):
        if len(args) == 1:
            a = args[0]
            x, y = a[0], a[1]
        elif len(args) == 2:
            x, y = args
        else:
            x, y = kw.get('x', 0.0), kw.get('y', 0.0)
        self.x = f32(x)
        self.y = f32(y)

    @staticmethod
    def _v(o):
        return o if isinstance(o, b2Vec2) else b2Vec2(o)

    def __add__(self, o):
        o = self._v(o)
        return b2Vec2(self.x + o.x, self.y + o.y)

    __radd__ = __add__

    def __sub__(self, o):
        o = self._v(o)
        return b2Vec2(self.x - o.x, self.y - o.y)

    def __rsub__(self, o):
        return self._v(o) - self

    def __mul__(self, a):
        a = f32(a)
        return b2Vec2(self.x * a, self.y * a)

    __rmul__ = __mul__

    def __neg__(self):
        return b2Vec2(-self.x, -self.y)

    def __getitem__(self, i):
        return float((self.x, self.y)[i])

    def __len__(self):
        return 2

    def __iter__(self):
        yield float(self.x)
        yield float(self.y)

    @property
    def length(self):
        return float(np.sqrt(self.x * self.x + self.y * self.y))

    @property
    def lengthSquared(self):
        return float(self.x * self.x + self.y * self.y)

    def copy(self):
        return b2Vec2(self.x, self.y)

    def _c(self):
        return _V2(self.x, self.y)

    def __repr__(self):
        return f'b2Vec2({float(self.x)}, {float(self.y)})'


class b2Mat22:
    def __init__(self, *args):
        self.ex = b2Vec2(1, 0)
        self.ey = b2Vec2(0, 1)
        if len(args) == 2:
            self.ex, self.ey = b2Vec2(args[0]), b2Vec2(args[1])

    @property
    def angle(self):
        return float(np.arctan2(self.ex.y, self.ex.x))

    @angle.setter
    def angle(self, a):
        s, c = _sincos(a)
        self.ex = b2Vec2(c, s)
        self.ey = b2Vec2(-s, c)

    def __mul__(self, v):
        v = b2Vec2._v(v)
        return b2Vec2(self.ex.x * v.x + self.ey.x * v.y, self.ex.y * v.x + self.ey.y * v.y)


class b2Transform:
    def __init__(self):
        self.position = b2Vec2(0, 0)
        self.s, self.c = f32(0.0), f32(1.0)

    def Set(self, position=(0, 0), angle=0.0):
        self.position = b2Vec2(position)
        self.s, self.c = _sincos(angle)

    @property
    def R(self):
        return b2Mat22(b2Vec2(self.c, self.s), b2Vec2(-self.s, self.c))

    @property
    def q(self):
        return self.R

    def _crot(self):
        return _Rot(self.s, self.c)


b2_staticBody = 0
b2_kinematicBody = 1
b2_dynamicBody = 2


class b2Shape:
    pass


class b2CircleShape(b2Shape):
    def __init__(self, radius=0.0, pos=(0, 0)):
        self.radius = float(f32(radius))
        self.pos = b2Vec2(pos)

    def TestPoint(self, transform, p):
        return bool(_L.ora_circle_test_point(c_float(self.radius), transform.position._c(), b2Vec2(p)._c()))

    def getAABB(self, transform, childIndex):
        return None


class b2PolygonShape(b2Shape):
    def __init__(self, box=None, vertices=None):
        self._p = _Poly()
        self.radius = float(f32(0.01))
        if box is not None:
            _L.ora_poly_set_as_box(byref(self._p), c_float(f32(box[0])), c_float(f32(box[1])))
        elif vertices is not None:
            vs = (_V2 * len(vertices))(*[_V2(f32(v[0]), f32(v[1])) for v in vertices])
            _L.ora_poly_set(byref(self._p), vs, len(vertices))

    @property
    def vertices(self):
        return [(float(self._p.v[i].x), float(self._p.v[i].y)) for i in range(self._p.count)]

    def TestPoint(self, transform, p):
        return bool(_L.ora_poly_test_point(byref(self._p), transform.position._c(), transform._crot(), b2Vec2(p)._c()))

    def getAABB(self, transform, childIndex):
        return None


class b2ChainShape(b2Shape):
    def __init__(self, vertices=None):
        self.vertices = vertices


class b2EdgeShape(b2Shape):
    def __init__(self, vertices=None):
        self.vertices = vertices


class b2FixtureDef:
    def __init__(self, shape=None, density=0.0, restitution=0.0, isSensor=False, friction=0.2):
        self.shape, self.density, self.restitution, self.isSensor = shape, density, restitution, isSensor


class b2Fixture:
    def __init__(self, body, fd):
        self.body = body
        self.shape = fd.shape  # Box2D clones the shape; shapes are never mutated here
        self.density = float(f32(fd.density))
        self.restitution = float(f32(fd.restitution))
        self.sensor = bool(fd.isSensor)


class b2Body:
    def __init__(self, world, type, position, angle, fixtures, linearDamping, angularDamping, userData):
        self.world = world
        self.type = type
        self._c = b2Vec2(position)
        self._a = f32(angle)
        self._v = b2Vec2(0, 0)
        self._w = f32(0.0)
        self._sleep = f32(0.0)
        self._awake = True
        self.linearDamping = float(f32(linearDamping))
        self.angularDamping = float(f32(angularDamping))
        self.userData = userData
        self.fixtures = [b2Fixture(self, fixtures)]
        self.serial = world._next_serial
        world._next_serial += 1
        shape = self.fixtures[0].shape
        if type == b2_dynamicBody and isinstance(shape, b2CircleShape):
            im, ii = c_float(), c_float()
            _L.ora_body_mass(c_float(shape.radius), c_float(self.fixtures[0].density), byref(im), byref(ii))
            self._inv_mass, self._inv_I = f32(im.value), f32(ii.value)
        else:
            self._inv_mass, self._inv_I = f32(0.0), f32(0.0)

    # pybox2d properties -------------------------------------------------
    @property
    def position(self):
        return self._c.copy()

    @property
    def worldCenter(self):
        return self._c.copy()

    @property
    def angle(self):
        return float(self._a)

    @property
    def linearVelocity(self):
        return self._v.copy()

    @property
    def angularVelocity(self):
        return float(self._w)

    @property
    def transform(self):
        t = b2Transform()
        t.position = self._c.copy()
        t.s, t.c = _sincos(self._a)
        return t

    def _wake(self):
        if not self._awake:
            self._awake = True
            self._sleep = f32(0.0)

    def ApplyLinearImpulse(self, impulse, point, wake=True):
        if self.type != b2_dynamicBody:
            return
        if wake:
            self._wake()
        if self._awake:
            J = b2Vec2._v(impulse)
            p = b2Vec2._v(point)
            self._v = self._v + J * self._inv_mass
            d = p - self._c
            self._w = f32(self._w + self._inv_I * (d.x * J.y - d.y * J.x))

    def ApplyAngularImpulse(self, impulse, wake=True):
        if self.type != b2_dynamicBody:
            return
        if wake:
            self._wake()
        if self._awake:
            self._w = f32(self._w + self._inv_I * f32(impulse))

    def __repr__(self):
        return f'b2Body#{self.serial}'


class b2RayCastCallback:
    def __init__(self):
        pass


class b2QueryCallback:
    def __init__(self):
        pass


class b2ContactListener:
    def __init__(self):
        pass


class b2Joint:
    pass


class b2AABB:
    def __init__(self, lowerBound=None, upperBound=None):
        self.lowerBound, self.upperBound = lowerBound, upperBound


def _is_solid_dynamic(b):
    return b.type == b2_dynamicBody and not b.fixtures[0].sensor


class b2World:
    def __init__(self, gravity=(0, 0), doSleep=True):
        self.bodies = []
        self._next_serial = 1
        self._inv_dt0 = 0.0
        self._cmem = {}  # (serialA, serialB) -> (touching, ni, ti)

    def CreateBody(self, type=b2_staticBody, position=(0, 0), angle=0.0, fixtures=None, linearDamping=0.0,
                   angularDamping=0.0, userData=None):
        b = b2Body(self, type, position, angle, fixtures, linearDamping, angularDamping, userData)
        self.bodies.append(b)
        return b

    def DestroyBody(self, body):
        if body in self.bodies:
            self.bodies.remove(body)
            s = body.serial
            self._cmem = {k: v for k, v in self._cmem.items() if s not in k}

    def ClearForces(self):
        pass

    # canonical fixture order ------------------------------------------
    def _canonical(self):
        alive = set(id(b) for b in self.bodies)
        out = []
        for g in CANONICAL_GROUPS:
            for b in g.bodies:
                if id(b) in alive:
                    out.append(b)
        return out

    def RayCast(self, callback, p1, p2):
        p1, p2 = b2Vec2._v(p1), b2Vec2._v(p2)
        maxf = f32(1.0)
        for b in self._canonical():
            sh = b.fixtures[0].shape
            fr = c_float()
            if isinstance(sh, b2CircleShape):
                hit = _L.ora_ray_circle(c_float(sh.radius), b._c._c(), p1._c(), p2._c(), c_float(maxf), byref(fr))
            else:
                t = b.transform
                hit = _L.ora_ray_poly(byref(sh._p), t.position._c(), t._crot(), p1._c(), p2._c(), c_float(maxf),
                                      byref(fr))
            if hit:
                f = f32(fr.value)
                point = p1 * (f32(1.0) - f) + p2 * f
                ret = f32(callback.ReportFixture(b.fixtures[0], point, b2Vec2(0, 0), float(f)))
                if ret == 0:
                    return
                if ret > 0:
                    maxf = ret

    def QueryAABB(self, callback, aabb):
        for b in self._canonical():
            if not callback.ReportFixture(b.fixtures[0]):
                return

    # physics ------------------------------------------------------------
    def Step(self, timeStep, velocityIterations, positionIterations):
        dyn = [b for b in self._canonical() if _is_solid_dynamic(b)]
        stat = []
        for g in STATIC_GROUPS:
            stat += [b for b in g.bodies if b in self.bodies]
        assert len(dyn) <= MAX_DYN and len(stat) <= MAX_STAT
        W = _World()
        W.n_dyn = len(dyn)
        if dyn:
            sh = dyn[0].fixtures[0].shape
            W.radius = f32(sh.radius)
            W.inv_mass = dyn[0]._inv_mass
            W.inv_I = dyn[0]._inv_I
            W.lin_damp = f32(dyn[0].linearDamping)
            W.ang_damp = f32(dyn[0].angularDamping)
        for i, b in enumerate(dyn):
            W.active[i] = 1
            W.c[i] = b._c._c()
            W.a[i] = b._a
            W.v[i] = b._v._c()
            W.w[i] = b._w
            W.sleep_time[i] = b._sleep
            W.awake[i] = int(b._awake)
        W.n_stat = len(stat)
        for k, b in enumerate(stat):
            W.sp[k] = b._c._c()
            W.sa[k] = b._a
            t = b.transform
            W.sq[k] = t._crot()
            W.spoly[k] = b.fixtures[0].shape._p
        for i, bi in enumerate(dyn):
            for j in range(i + 1, len(dyn)):
                m = self._cmem.get((bi.serial, dyn[j].serial))
                if m:
                    W.aa[i][j] = _Cmem(*m)
            for k, bs in enumerate(stat):
                m = self._cmem.get((bs.serial, bi.serial))
                if m:
                    W.as_[i][k] = _Cmem(*m)
        W.inv_dt0 = f32(self._inv_dt0)
        _L.ora_world_step(byref(W), c_float(f32(timeStep)), velocityIterations, positionIterations)
        self._inv_dt0 = float(W.inv_dt0)
        for i, b in enumerate(dyn):
            b._c = b2Vec2(W.c[i].x, W.c[i].y)
            b._a = f32(W.a[i])
            b._v = b2Vec2(W.v[i].x, W.v[i].y)
            b._w = f32(W.w[i])
            b._sleep = f32(W.sleep_time[i])
            b._awake = bool(W.awake[i])
        for i, bi in enumerate(dyn):
            for j in range(i + 1, len(dyn)):
                m = W.aa[i][j]
                self._cmem[(bi.serial, dyn[j].serial)] = (m.touching, m.ni, m.ti)
            for k, bs in enumerate(stat):
                m = W.as_[i][k]
                self._cmem[(bs.serial, bi.serial)] = (m.touching, m.ni, m.ti)
