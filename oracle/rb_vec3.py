"""Restatement of ``Fast4DMatrix::Vec3`` — TEST INFRASTRUCTURE ONLY.

Follows ``ext/fast_4d_matrix/fast_4d_matrix.c`` (the reference's only native
code), compiled there with ``-O3 -msse2 -mavx`` and no ``-ffast-math``/FMA
(``extconf.rb:6-10``): strict IEEE doubles, left-to-right sums.  Python floats
are IEEE doubles with no contraction, so every operation below is bit-identical
to the C extension's.

Semantics that matter:
* ``r`` is ``sqrt(x*x + y*y + z*z)`` fixed at creation (``:62-73``); ``r2`` is
  ``r*r`` (``:280-284``), *not* ``x*x + y*y + z*z``.
* ``dot`` accumulates from ``0.0`` (``:100-106``).
* ``cos`` is ``sqrt(dot*dot / |a|^2 / |b|^2)`` clamped to <= 1, i.e. **|cos|**,
  and raises on a zero vector (``:109-129``).
* ``normalize`` recomputes the norm and raises on zero (``:286-293``).
* ``*`` is scalar or component-wise (``:190-208``); ``/`` is scalar only
  (``:209-224``).
"""

import math


class RtxError(Exception):
    """A reference raise site; ``kind`` in {'zero_vec', 'color_gt1', 'domain', 'type'}."""

    def __init__(self, kind, msg):
        super().__init__(msg)
        self.kind = kind


class Vec3:
    __slots__ = ("x", "y", "z", "r")

    def __init__(self, x, y, z):
        # Vec3_c_create / from_a (fast_4d_matrix.c:62-83)
        self.x = x
        self.y = y
        self.z = z
        self.r = math.sqrt(x * x + y * y + z * z)

    @classmethod
    def from_a(cls, x, y, z):
        return cls(float(x), float(y), float(z))

    def to_a(self):
        return [self.x, self.y, self.z]

    @property
    def r2(self):
        return self.r * self.r

    def dot(self, o):
        ret = 0.0
        ret += self.x * o.x
        ret += self.y * o.y
        ret += self.z * o.z
        return ret

    def cos(self, o):
        ret = 0.0
        ret += self.x * o.x
        ret += self.y * o.y
        ret += self.z * o.z
        r1 = self.x * self.x + self.y * self.y + self.z * self.z
        r2 = o.x * o.x + o.y * o.y + o.z * o.z
        if r1 == 0 or r2 == 0:
            raise RtxError("zero_vec", "zero vector detected!")
        v = math.sqrt(ret * ret / r1 / r2)
        if v > 1:
            v = 1.0
        return v

    def cross(self, o):
        return Vec3(self.y * o.z - self.z * o.y,
                    self.z * o.x - self.x * o.z,
                    self.x * o.y - self.y * o.x)

    def __add__(self, o):
        return Vec3(self.x + o.x, self.y + o.y, self.z + o.z)

    def __sub__(self, o):
        return Vec3(self.x - o.x, self.y - o.y, self.z - o.z)

    def __mul__(self, o):
        if isinstance(o, Vec3):
            return Vec3(self.x * o.x, self.y * o.y, self.z * o.z)
        o = float(o)
        return Vec3(self.x * o, self.y * o, self.z * o)

    def __truediv__(self, o):
        if isinstance(o, Vec3):
            raise TypeError("parameter must be float")   # fast_4d_matrix.c:220
        o = float(o)
        return Vec3(self.x / o, self.y / o, self.z / o)

    def __neg__(self):
        return Vec3(-self.x, -self.y, -self.z)

    def __pos__(self):
        return Vec3(self.x, self.y, self.z)

    # in-place forms recompute the cached r (Vec3_c_recalc_r, :226-273)
    def add_bang(self, o):
        self.__init__(self.x + o.x, self.y + o.y, self.z + o.z)
        return self

    def sub_bang(self, o):
        self.__init__(self.x - o.x, self.y - o.y, self.z - o.z)
        return self

    def mul_bang(self, o):
        if isinstance(o, Vec3):
            self.__init__(self.x * o.x, self.y * o.y, self.z * o.z)
        else:
            o = float(o)
            self.__init__(self.x * o, self.y * o, self.z * o)
        return self

    def normalize(self):
        r = math.sqrt(self.x * self.x + self.y * self.y + self.z * self.z)
        if r == 0:
            raise RtxError("zero_vec", "zero vector detected")
        return Vec3(self.x / r, self.y / r, self.z / r)

    # lib/fast_4d_matrix/fast_4d_matrix.rb:7-13
    def to_s(self, n=6):
        if n:
            return "[" + ", ".join(("%0." + str(n) + "f") % v for v in self.to_a()) + "]"
        return str(self.to_a())

    def __repr__(self):
        return "Vec3(%r, %r, %r)" % (self.x, self.y, self.z)
