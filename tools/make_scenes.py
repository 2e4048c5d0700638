#!/usr/bin/env python3
"""Generate the committed benchmark/parity scenes and their
synthetic textures.  Deterministic (numpy RandomState with fixed seeds).

  scenes/c0_world.yml  default world of the reference (config/world.yml restated),
                       the missing ./textures/floor.jpg replaced by a synthetic
                       checker; the front wall's texture is the reference's own
                       textures/RubyOnRails.png (122x158, 16-bit RGBA), copied
                       as data into scenes/textures/
  scenes/c1_world.yml  1 sphere + ground plane + point light
  scenes/c2_world.yml  64 spheres (jittered 8x8 grid) + ground + area light
  scenes/c4_world.yml  4096 random spheres + ground textured with RubyOnRails.png
                        + area light
  scenes/cN_camera.yml the reference camera (config/camera.yml) with the
                       config's size / samples / depth
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raytracing_rb_amd import png  # noqa: E402

SC = os.path.join(ROOT, "scenes")


def f(v):
    return repr(float(v))


def vec(v):
    return "[%s]" % ", ".join(f(x) for x in v)


def textures():
    os.makedirs(os.path.join(SC, "textures"), exist_ok=True)
    # floor: 64x64 8-bit RGB checker of 8x8 cells, two wood-ish tones
    yy, xx = np.mgrid[0:64, 0:64]
    c = ((xx // 8 + yy // 8) % 2).astype(np.uint8)
    img = np.where(c[..., None] == 1, np.array([200, 170, 120], np.uint8), np.array([90, 60, 40], np.uint8))
    png.write(os.path.join(SC, "textures", "checker.png"), img)
    # rails_synth: 122x158 16-bit RGBA (same shape/format as the reference's
    # RubyOnRails.png): white field, red disc, dark stripes, smooth gradient.
    h, w = 158, 122
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    r = np.full((h, w), 65535.0)
    g = np.full((h, w), 65535.0)
    b = np.full((h, w), 65535.0)
    disc = (xx - 61) ** 2 + (yy - 60) ** 2 < 45 ** 2
    r[disc], g[disc], b[disc] = 52000, 4000, 6000
    stripe = (yy > 115) & (((xx // 6) % 2) == 0)
    r[stripe], g[stripe], b[stripe] = 9000, 9000, 12000
    g = np.minimum(g, 65535 - yy * 120)
    rgba = np.stack([r, g, b, np.full((h, w), 65535.0)], axis=2).astype(np.uint16)
    png.write(os.path.join(SC, "textures", "rails_synth.png"), rgba)


CAMERA = """position:         [0.0, 0.0, 0.0]
up:               [0.0, 0.0, 1.0]
front:            [1.0, 0.0, 0.0]
retina_width:     0.016
retina_height:    0.009
aperture_radius:  0.001
image_distance:   0.01714573877962683
focal_distance:   0.017
width:            {w}
height:           {h}
pre_sample_times: {pre}
max_sample_times: {mx}
variant_threshold: 0.001
trace_depth:      {d}
monte_carlo_diffusion_times: 1
"""


def camera(name, w, h, pre, mx, d):
    with open(os.path.join(SC, name), "w") as fh:
        fh.write("# %s\n" % name + CAMERA.format(w=w, h=h, pre=pre, mx=mx, d=d))


C0 = """# Default world of the reference (config/world.yml), restated.  The ground
# texture ./textures/floor.jpg is missing from the reference repo and is
# replaced by a synthetic checker; RubyOnRails.png is the reference's own file.
# The front wall keeps the duplicate keys (YAML: last wins).
max_distance:           10000
soft_shadow_exponent:   2
lights:
  - type: Spot
    properties:
      name:             Main
      position:         [5, -4, 0.9]
      radius:           0.8
      color:            [1, 1, 1]
      high_light_rate:  1
      high_light_angle: 3
world_objects:
  - type: Plane
    properties:
      name:                     ground
      point:                    [0, 0, -1]
      front:                    [0, 0, 1]
      up:                       [1, 0, 0]
      u_unit:                   1
      v_unit:                   1
      specular_power:           3
      specular_rate:            [0.2, 0.2, 0.2]
      diffuse_rate:             [0.6, 0.6, 0.6]
      reflective_attenuation:   [0.39, 0.39, 0.39]
      ambient:                  [0.01, 0.01, 0.01]
      texture_file_path:        ./textures/checker.png
      texture_horizontal_scale: 0.01
      texture_vertical_scale:   0.06
  - type: Plane
    properties:
      name:                     front wall
      point:                    [15, 0, 0]
      front:                    [-1, 0, 0]
      up:                       [0, 0, -1]
      diffuse_rate:             [0.4, 0.4, 0.4]
      reflective_attenuation:   [0.3, 0.3, 0.3]
      ambient:                  [0.1, 0.1, 0.1]
      u_unit:                   1
      v_unit:                   1
      specular_power:           3
      specular_rate:            [0.2, 0.2, 0.2]
      diffuse_rate:             [0.6, 0.6, 0.6]
      reflective_attenuation:   [0.39, 0.39, 0.39]
      ambient:                  [0.01, 0.01, 0.01]
      texture_file_path:        ./textures/RubyOnRails.png
      texture_horizontal_scale: 0.015
      texture_vertical_scale:   0.015
  - type: Sphere
    properties:
      name:                     small sphere
      center:                   [5, -2, -0.3]
      radius:                   0.7
      refractive_rate:          1.6
      reflective_attenuation:   [0.1, 0.1, 0.1]
      refractive_attenuation:   [0.8, 0.8, 0.8]
      diffuse_rate:             [0.09, 0.09, 0.09]
      ambient:                  [0.01, 0.01, 0.01]
"""

GROUND = """  - type: Plane
    properties:
      name:                   ground
      point:                  [0.0, 0.0, -1.0]
      front:                  [0.0, 0.0, 1.0]
      up:                     [1.0, 0.0, 0.0]
      diffuse_rate:           [0.6, 0.6, 0.6]
      reflective_attenuation: [0.3, 0.3, 0.3]
      ambient:                [0.05, 0.05, 0.05]
{extra}"""


def sphere(name, c, r, mat):
    d, a, rl, rr = mat
    return ("  - type: Sphere\n    properties:\n"
            "      name:                   %s\n"
            "      center:                 %s\n"
            "      radius:                 %s\n"
            "      refractive_rate:        1.5\n"
            "      diffuse_rate:           %s\n"
            "      ambient:                %s\n"
            "      reflective_attenuation: %s\n"
            "      refractive_attenuation: %s\n") % (name, vec(c), f(r), vec(d), vec(a), vec(rl), vec(rr))


def material(rs, kind):
    """diffuse / mirror / glass; per-channel d + a + refl + refr <= 0.98 (rt_reduce never raises)."""
    if kind == 0:      # diffuse, coloured
        d = rs.uniform(0.25, 0.7, 3)
        return d, [0.02] * 3, [0.1] * 3, [0.0] * 3
    if kind == 1:      # mirror
        d = rs.uniform(0.02, 0.1, 3)
        return d, [0.01] * 3, [0.8] * 3, [0.0] * 3
    d = rs.uniform(0.02, 0.06, 3)   # glass
    return d, [0.01] * 3, [0.1] * 3, [0.8] * 3


def light(pos, radius):
    return ("lights:\n  - type: Spot\n    properties:\n"
            "      name:             Main\n"
            "      position:         %s\n"
            "      radius:           %s\n"
            "      color:            [1.0, 1.0, 1.0]\n"
            "      high_light_rate:  1.0\n"
            "      high_light_angle: 3.0\n") % (vec(pos), f(radius))


def kinds(rs, n):
    k = np.array([0] * (n // 2) + [1] * (n // 4) + [2] * (n - n // 2 - n // 4))
    rs.shuffle(k)
    return k


def c1():
    s = ("# C1: 1 sphere + ground plane + point light (SURVEY.md 8d)\n"
         "max_distance:           10000\nsoft_shadow_exponent:   2\n")
    s += light([2.0, -3.0, 4.0], 0.0)
    s += "world_objects:\n"
    s += sphere("ball", [5.0, 0.0, 0.0], 1.0, ([0.5] * 3, [0.05] * 3, [0.3] * 3, [0.0] * 3))
    s += GROUND.format(extra="")
    return s


def c2():
    rs = np.random.RandomState(2024)
    s = ("# C2: 64 spheres on a jittered 8x8 grid + ground + area light (SURVEY.md 8d)\n"
         "max_distance:           10000\nsoft_shadow_exponent:   2\n")
    s += light([6.0, -4.0, 5.0], 0.8)
    s += "world_objects:\n"
    k = kinds(rs, 64)
    i = 0
    for gx in range(8):
        for gy in range(8):
            r = rs.uniform(0.2, 0.45)
            x = 4.0 + gx + rs.uniform(0.05, 0.95)
            y = -4.0 + gy + rs.uniform(0.05, 0.95)
            s += sphere("s%02d" % i, [x, y, -1.0 + r], r, material(rs, k[i]))
            i += 1
    s += GROUND.format(extra="")
    return s


C4_HEADER = "# C4: 4096 random spheres + ground textured with RubyOnRails.png + area light (SURVEY.md 8d)"


def c4():
    rs = np.random.RandomState(4096)
    s = (C4_HEADER + "\n"
         "max_distance:           10000\nsoft_shadow_exponent:   2\n")
    s += light([10.0, -6.0, 12.0], 1.0)
    s += "world_objects:\n"
    k = kinds(rs, 4096)
    for i in range(4096):
        c = [rs.uniform(3, 40), rs.uniform(-20, 20), rs.uniform(-1, 8)]
        r = rs.uniform(0.05, 0.3)
        s += sphere("s%04d" % i, c, r, material(rs, k[i]))
    s += GROUND.format(extra=("      u_unit:                 1\n"
                              "      v_unit:                 1\n"
                              "      texture_file_path:      ./textures/RubyOnRails.png\n"
                              "      texture_horizontal_scale: 0.015\n"
                              "      texture_vertical_scale: 0.015\n"))
    return s


def ensure_c4():
    """scenes/c4_world.yml is generated (2 MB, not committed): write it if missing
    or from an older generator (its first line)."""
    path = os.path.join(SC, "c4_world.yml")
    current = False
    if os.path.exists(path):
        with open(path) as fh:
            current = fh.readline().rstrip("\n") == C4_HEADER
    if not current:
        tmp = path + ".%d.tmp" % os.getpid()
        with open(tmp, "w") as fh:
            fh.write(c4())
        os.replace(tmp, path)
    return path


def main():
    os.makedirs(SC, exist_ok=True)
    textures()
    for name, body in (("c0_world.yml", C0), ("c1_world.yml", c1()), ("c2_world.yml", c2()),
                       ("c4_world.yml", c4())):
        with open(os.path.join(SC, name), "w") as fh:
            fh.write(body)
    camera("camera.yml", 192, 108, 3, 10, 4)            # config/camera.yml as shipped
    camera("c0_camera.yml", 320, 240, 1, 1, 1)
    camera("c1_camera.yml", 1920, 1080, 1, 1, 1)
    camera("c2_camera.yml", 1920, 1080, 4, 4, 5)
    camera("c4_camera.yml", 3840, 2160, 8, 8, 8)


if __name__ == "__main__":
    main()
