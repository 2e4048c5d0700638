"""Seeded random scenes for the fuzz parity tests (test_oracle.py on the CPU,
test_gpu_fuzz.py on the GPU): every object kind and material path of the
reference (Sphere / Plane / Box, textured spheres and planes, mirrors, glass,
refractive planes, point and area lights, path tracing), random camera
sampling (pre / max samples, variance threshold), depth and
soft_shadow_exponent.  Written as world.yml / camera.yml files in the
reference's schema, so both restatements and the product load them through
their own loaders."""

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TEXTURES = os.path.join(os.path.dirname(HERE), "scenes", "textures")


def _v(a):
    return "[%s]" % ", ".join(repr(float(x)) for x in a)


def _material(rs, kind):
    """(diffuse, ambient, reflective, refractive) attenuations of a material kind."""
    if kind == "diffuse":
        return rs.uniform(0.2, 0.8, 3), rs.uniform(0.0, 0.06, 3), rs.uniform(0.0, 0.15, 3), [0.0, 0.0, 0.0]
    if kind == "mirror":
        return rs.uniform(0.02, 0.1, 3), rs.uniform(0.0, 0.02, 3), rs.uniform(0.5, 0.9, 3), [0.0, 0.0, 0.0]
    return rs.uniform(0.02, 0.1, 3), rs.uniform(0.0, 0.02, 3), rs.uniform(0.05, 0.2, 3), rs.uniform(0.5, 0.9, 3)


def make(seed, out_dir, width=40, height=24):
    rs = np.random.RandomState(seed)
    lines = ["max_distance: 10000", "soft_shadow_exponent: %d" % int(rs.choice([1, 2, 3])), "lights:"]
    for k in range(rs.randint(1, 4)):
        radius = 0.0 if rs.rand() < 0.3 else rs.uniform(0.2, 1.0)
        lines += ["  - type: Spot", "    properties:", "      name: l%d" % k,
                  "      position: %s" % _v([rs.uniform(2, 10), rs.uniform(-6, 6), rs.uniform(3, 9)]),
                  "      radius: %r" % float(radius),
                  "      color: %s" % _v(rs.uniform(0.4, 1.0, 3)),
                  "      high_light_rate: %r" % float(rs.uniform(0.3, 1.0)),
                  "      high_light_angle: %r" % float(rs.uniform(0.5, 4.0))]
    lines.append("world_objects:")
    # ground plane, optionally textured, optionally refractive (a glass floor)
    d, a, rl, rr = _material(rs, "diffuse")
    lines += ["  - type: Plane", "    properties:", "      name: ground",
              "      point: [0.0, 0.0, %r]" % float(rs.uniform(-1.5, -0.5)),
              "      front: [0.0, 0.0, 1.0]", "      up: [1.0, 0.0, 0.0]",
              "      diffuse_rate: %s" % _v(d), "      ambient: %s" % _v(a),
              "      reflective_attenuation: %s" % _v(rl)]
    if rs.rand() < 0.5:
        lines += ["      u_unit: %r" % float(rs.uniform(0.5, 2.0)), "      v_unit: %r" % float(rs.uniform(0.5, 2.0)),
                  "      texture_file_path: %s" % os.path.join(TEXTURES, "checker.png"),
                  "      texture_horizontal_scale: %r" % float(rs.uniform(0.01, 0.05)),
                  "      texture_vertical_scale: %r" % float(rs.uniform(0.01, 0.05))]
    if rs.rand() < 0.25:
        lines += ["      refractive_rate: %r" % float(rs.uniform(1.1, 1.6)),
                  "      refractive_attenuation: %s" % _v(rs.uniform(0.1, 0.5, 3))]
    # spheres: diffuse / mirror / glass, some textured, some overlapping
    for k in range(rs.randint(3, 40)):
        kind = rs.choice(["diffuse", "mirror", "glass"], p=[0.5, 0.3, 0.2])
        d, a, rl, rr = _material(rs, kind)
        lines += ["  - type: Sphere", "    properties:", "      name: s%d" % k,
                  "      center: %s" % _v([rs.uniform(3, 14), rs.uniform(-5, 5), rs.uniform(-0.8, 3.0)]),
                  "      radius: %r" % float(rs.uniform(0.15, 1.3)),
                  "      refractive_rate: %r" % float(rs.uniform(1.1, 1.8)),
                  "      diffuse_rate: %s" % _v(d), "      ambient: %s" % _v(a),
                  "      reflective_attenuation: %s" % _v(rl), "      refractive_attenuation: %s" % _v(rr)]
        if kind == "diffuse" and rs.rand() < 0.3:
            lines += ["      north_pole_vec: [0, 0, 1]", "      greenwich_vec: [-1, 0, 0]",
                      "      texture_file_path: %s" % os.path.join(TEXTURES, "rails_synth.png"),
                      "      texture_horizontal_scale: %r" % float(rs.uniform(0.002, 0.01)),
                      "      texture_vertical_scale: %r" % float(rs.uniform(0.002, 0.01)),
                      "      texture_u_offset: %r" % float(rs.uniform(0, 0.5)),
                      "      texture_v_offset: %r" % float(rs.uniform(0, 0.5))]
    # boxes (box.rb): random orientation about z
    for k in range(rs.randint(0, 3)):
        th = rs.uniform(0, np.pi)
        d, a, rl, rr = _material(rs, "diffuse")
        lines += ["  - type: Box", "    properties:", "      name: b%d" % k,
                  "      point: %s" % _v([rs.uniform(5, 12), rs.uniform(-4, 4), rs.uniform(-0.5, 1.5)]),
                  "      front: %s" % _v([np.cos(th), np.sin(th), 0.0]), "      up: [0.0, 0.0, 1.0]",
                  "      width_front: %r" % float(rs.uniform(0.3, 1.5)), "      width_up: %r" % float(rs.uniform(0.3, 1.5)),
                  "      width_left: %r" % float(rs.uniform(0.3, 1.5)),
                  "      diffuse_rate: %s" % _v(d), "      ambient: %s" % _v(a),
                  "      reflective_attenuation: %s" % _v(rl)]
    pre = int(rs.randint(1, 5))
    cam = ["position: [0.0, 0.0, 0.0]", "up: [0.0, 0.0, 1.0]", "front: [1.0, 0.0, 0.0]",
           "retina_width: 0.016", "retina_height: %r" % float(0.016 * height / width),
           "aperture_radius: %r" % float(rs.choice([0.0, 0.0005, 0.002])),
           "image_distance: 0.01714573877962683", "focal_distance: 0.017",
           "width: %d" % width, "height: %d" % height,
           "pre_sample_times: %d" % pre, "max_sample_times: %d" % (pre + int(rs.randint(0, 4))),
           "variant_threshold: %r" % float(rs.choice([0.0, 0.0005, 0.01, 1e9])),
           "trace_depth: %d" % rs.randint(1, 7), "monte_carlo_diffusion_times: %d" % rs.randint(1, 4)]
    w = os.path.join(str(out_dir), "fuzz%d_world.yml" % seed)
    c = os.path.join(str(out_dir), "fuzz%d_camera.yml" % seed)
    with open(w, "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(c, "w") as f:
        f.write("\n".join(cam) + "\n")
    return w, c
