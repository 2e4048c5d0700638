"""Search for Sphere#cover_area inputs whose Math.acos raises (sphere.rb:42-46).

In exact arithmetic cos_theta1 and cos_theta2 of Sphere#cover_area cannot go
below -1 inside the branch d > |R - r1|:

    cos_theta1 + 1 = (r1 + d - R)(r1 + d + R) / (2 r1 d)
    cos_theta2 + 1 = (R + d - r1)(R + d + r1) / (2 R d)

but rounded they can, when d (the sphere center's distance from the line
target -> light) lies within a few ulps of |R - r1|.  This script places a
sphere at that tangency for a given target T, light L and light radius, with
random jitter, and keeps the first placement whose cover_area (evaluated with
the reference's operations in binary64, the order of rt_oracle.c) raises:

  regime "A": R > r1, the center at distance R - r1 from the line (the line
              crosses the sphere); `side` < 0 puts it behind T (binary cover
              factor 0: the shading walks never evaluate its penumbra);
  regime "B": r1 > R, the sphere inside the cone of half-slope radius/|L - T|
              touching it from inside (the line misses the sphere).

    python tools/raise_search.py          # prints the configurations the tests use

Test infrastructure: the found spheres are committed in
tests/golden/raise_scenes.json (tests/test_raises.py re-runs this search on
CPU and checks it reproduces them).
"""

import json
import math
import random
import sys


def _sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def _add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def _sc(a, s):
    return (a[0] * s, a[1] * s, a[2] * s)


def _dot(a, b):                     # fast_4d_matrix.c:98-107: accumulated from 0
    s = 0.0
    s += a[0] * b[0]
    s += a[1] * b[1]
    s += a[2] * b[2]
    return s


def _r(a):                          # :62-73
    return math.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])


def _r2(a):                         # :280-284: r, squared
    x = _r(a)
    return x * x


def cover_raises(C, R, T, L, radius):
    """The acos arguments of Sphere#cover_area(L, radius, T) (sphere.rb:31-46):
    returns (cos_theta1, cos_theta2) when the acos branch runs, else None."""
    lt = _sub(L, T)
    t = _dot(_sub(C, T), lt) / _r2(lt)
    x1 = _add(T, _sc(lt, t))
    r1 = radius * (_r(_sub(x1, T)) / _r(lt))
    d = _r(_sub(x1, C))
    if d >= r1 + R:
        return None
    if d > abs(R - r1):
        return (min((r1 * r1 + d * d - R * R) / (2 * r1 * d), 1.0),
                min((R * R + d * d - r1 * r1) / (2 * R * d), 1.0))
    return None


def find_sphere(T, L, radius, regime="A", side=-1.0, seed=1, tries=200000, s_range=(0.5, 3.0), r_range=(0.05, 0.5)):
    """A sphere (C, R) whose cover_area from T towards L raises; `side` the
    sign of its center's position along T -> L (A only; B uses side too);
    r_range: B's radius as a fraction of the cone's r1 there (below 0.5 the
    line misses the sphere, so its binary cover factor is 0)."""
    rng = random.Random(seed)
    lt = _sub(L, T)
    n = _r(lt)
    u = _sc(lt, 1.0 / n)
    # a unit vector perpendicular to the axis
    a = (1.0, 0.0, 0.0) if abs(u[0]) < 0.9 else (0.0, 1.0, 0.0)
    p = _sub(a, _sc(u, _dot(a, u)))
    p = _sc(p, 1.0 / _r(p))
    k = radius / n
    for i in range(tries):
        s = side * rng.uniform(*s_range)
        r1 = k * abs(s)
        if regime == "A":
            R = r1 + rng.uniform(0.05, 1.0)
            rho = R - r1
        else:
            R = rng.uniform(*r_range) * r1
            rho = r1 - R
        C = _add(T, _add(_sc(u, s), _sc(p, rho)))
        c = cover_raises(C, R, T, L, radius)
        if c and (c[0] < -1 or c[1] < -1):
            return {"center": list(C), "radius": R, "tries": i + 1, "cos": list(c)}
    return None


# The configurations the tests use (tests/golden/raise_scenes.json):
#   highlight: camera (aperture 0) at T looking at the light; the raising
#              sphere behind the camera.  Every camera ray in the highlight
#              cone evaluates lit_area(T, L, radius) and raises.
#   shadow_A / shadow_B: target T = hit + delta of the ray (0,0,1) -> (0,0,-1)
#              on the plane z = 0 (hit (0,0,0), delta (0,0,1e-5)); the light
#              off the reflection's cone; spheres below the plane (A) or
#              beside the cone (B).
#   pixel_*:   T = hit + delta of one camera pixel's primary ray on the plane
#              z = 0 (PIXEL_CAMERA, pixel (9, 5); computed with the reference's
#              operations by tests/golden/make_raise_scenes.py, which passes it
#              in as `pixel_T`), so a whole render raises at that pixel: behind
#              T (A), inside the cone between T and the light with the line
#              missing the sphere (B), beyond the light (A).
CASES = {
    "highlight": dict(T=(0.0, 0.0, 0.0), L=(6.0, 0.5, 0.25), radius=0.8, regime="A", side=-1.0, seed=11),
    "shadow_A": dict(T=(0.0, 0.0, 1e-05), L=(3.0, 0.0, 4.0), radius=0.8, regime="A", side=-1.0, seed=12),
    "shadow_B": dict(T=(0.0, 0.0, 1e-05), L=(3.0, 0.0, 4.0), radius=2.5, regime="B", side=-1.0, seed=13,
                     s_range=(2.0, 4.0)),
    "pixel_A_back": dict(T=None, L=(3.0, 0.0, 4.0), radius=0.8, regime="A", side=-1.0, seed=21),
    "pixel_B_front": dict(T=None, L=(3.0, 0.0, 4.0), radius=1.5, regime="B", side=1.0, seed=22,
                          s_range=(1.5, 4.0), r_range=(0.05, 0.45)),
    "pixel_A_far": dict(T=None, L=(3.0, 0.0, 4.0), radius=0.8, regime="A", side=1.0, seed=23,
                        s_range=(7.5, 9.5)),
}
PIXEL = (9, 5)
PIXEL_CAMERA = dict(position=(-1.0, -4.0, 3.0), front=(1.0, 4.0, -3.0), width=24, height=16)


def search_all(pixel_T=None):
    """Every configuration; the pixel cases need their T (pixel_T: the
    reference-arithmetic hit + delta of PIXEL, computed by the caller)."""
    out = {}
    for name, c in CASES.items():
        kw = dict(c)
        T, L, radius = kw.pop("T"), kw.pop("L"), kw.pop("radius")
        if T is None:
            if pixel_T is None:
                continue
            T = tuple(pixel_T)
        f = find_sphere(T, L, radius, **kw)
        if f is None:
            raise RuntimeError("no raising configuration found for %s" % name)
        out[name] = dict(T=list(T), L=list(L), light_radius=radius, **f)
    return out


if __name__ == "__main__":
    res = search_all()
    json.dump(res, sys.stdout, indent=1)
    print()
