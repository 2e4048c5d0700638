"""``Fast4DMatrix::Vec3`` over the C-ABI (``rtx_vec3_*`` in librtx).

The API surface of the reference's native module
(``ext/fast_4d_matrix/fast_4d_matrix.c:29-55`` + the Ruby side
``lib/fast_4d_matrix/fast_4d_matrix.rb``): ``from_a, to_a, to_s, r, r2, dot,
cos, cross, + - * /, add! sub! mul! (add_bang ...), +@ -@, normalize,
normalize!``.  Every operation is computed by librtx with the C extension's
arithmetic (cached ``r``, ``r2 = r*r``, ``|cos|``, zero-vector errors).
"""

import ctypes as C
import json

from ._abi import Vec3T, load_library


class ZeroVectorError(RuntimeError):
    pass


def _lib():
    return load_library()


class Vec3:
    __slots__ = ("_v",)

    def __init__(self, x=0.0, y=0.0, z=0.0, _raw=None):
        self._v = _raw if _raw is not None else _lib().rtx_vec3_from_a(float(x), float(y), float(z))

    @classmethod
    def from_a(cls, x, y, z):                           # fast_4d_matrix.c:75-84
        return cls(x, y, z)

    @classmethod
    def _wrap(cls, raw):
        return cls(_raw=raw)

    def to_a(self):
        return [self._v.v[0], self._v.v[1], self._v.v[2]]

    def to_s(self, n=6):                                # fast_4d_matrix.rb:7-13
        if n:
            return "[" + ", ".join(("%0." + str(n) + "f") % v for v in self.to_a()) + "]"
        return str(self.to_a())

    def to_json(self):                                  # fast_4d_matrix.rb:27
        return json.dumps(self.to_a())

    @property
    def r(self):
        return _lib().rtx_vec3_r(self._v)

    @property
    def r2(self):
        return _lib().rtx_vec3_r2(self._v)

    def dot(self, o):
        return _lib().rtx_vec3_dot(self._v, o._v)

    def cos(self, o):
        out = C.c_double()
        if _lib().rtx_vec3_cos(self._v, o._v, C.byref(out)):
            raise ZeroVectorError("zero vector detected!")
        return out.value

    def cross(self, o):
        return Vec3._wrap(_lib().rtx_vec3_cross(self._v, o._v))

    def __add__(self, o):
        return Vec3._wrap(_lib().rtx_vec3_add(self._v, o._v))

    def __sub__(self, o):
        return Vec3._wrap(_lib().rtx_vec3_sub(self._v, o._v))

    def __mul__(self, o):                               # Float or Vec3 (:190-208)
        if isinstance(o, Vec3):
            return Vec3._wrap(_lib().rtx_vec3_mul(self._v, o._v))
        return Vec3._wrap(_lib().rtx_vec3_scale(self._v, float(o)))

    def __truediv__(self, o):                           # Float only (:209-224)
        if isinstance(o, Vec3):
            raise TypeError("parameter must be float")
        return Vec3._wrap(_lib().rtx_vec3_div(self._v, float(o)))

    def __neg__(self):
        return Vec3._wrap(_lib().rtx_vec3_neg(self._v))

    def __pos__(self):
        return Vec3._wrap(_lib().rtx_vec3_pos(self._v))

    def normalize(self):
        out = Vec3T()
        if _lib().rtx_vec3_normalize(self._v, C.byref(out)):
            raise ZeroVectorError("zero vector detected")
        return Vec3._wrap(out)

    # in-place forms (:230-273, :294-305)
    def add_bang(self, o):
        self._v = _lib().rtx_vec3_add_bang(self._v, o._v)
        return self

    def sub_bang(self, o):
        self._v = _lib().rtx_vec3_sub_bang(self._v, o._v)
        return self

    def mul_bang(self, o):
        if isinstance(o, Vec3):
            self._v = _lib().rtx_vec3_mul_bang(self._v, o._v)
        else:
            self._v = _lib().rtx_vec3_mul_bang_scalar(self._v, float(o))
        return self

    def normalize_bang(self):
        n = self.normalize()
        self._v = n._v
        self._v.r = 1.0                                 # normalize! sets r = 1 (:294-305)
        return self

    def __repr__(self):
        return "Vec3(%r, %r, %r)" % tuple(self.to_a())
