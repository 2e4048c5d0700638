"""Test infrastructure for tests/test_raises.py: the target point T of the
pixel cases of tools/raise_search.py (PIXEL_CAMERA's primary ray through
PIXEL hits the plane z = 0; T = intersection + delta, the point World#local_lights
is called with, ray_tracer.rb:115), computed by the Python restatement of the
reference (oracle/rt_ref.py: Camera#lens_func camera.rb:129-151, Plane#intersect
plane.rb:38-51), so a render of that camera meets exactly this T."""

import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import raise_search  # noqa: E402

PLANE = """  - type: Plane
    properties:
      name: ground
      point: [0.0, 0.0, 0.0]
      front: [0.0, 0.0, 1.0]
      up: [1.0, 0.0, 0.0]
      diffuse_rate: [0.6, 0.6, 0.6]
      reflective_attenuation: [0.3, 0.3, 0.3]
      ambient: [0.05, 0.05, 0.05]
"""


def vec(a):
    return "[%s]" % ", ".join(repr(float(x)) for x in a)


def camera_yaml(position, front, w, h, depth=2):
    return """position: %s
up: [0.0, 0.0, 1.0]
front: %s
retina_width: 0.016
retina_height: 0.012
aperture_radius: 0.0
image_distance: 0.0171
focal_distance: 0.017
width: %d
height: %d
pre_sample_times: 1
max_sample_times: 1
variant_threshold: 0.001
trace_depth: %d
monte_carlo_diffusion_times: 1
""" % (vec(position), vec(front), w, h, depth)


def pixel_T():
    from oracle import rt_ref
    cam_cfg = raise_search.PIXEL_CAMERA
    world = ("max_distance: 10000\nsoft_shadow_exponent: 2\nlights:\n  - type: Spot\n    properties:\n"
             "      name: L\n      position: [3.0, 0.0, 4.0]\n      radius: 0.8\n      color: [0.5, 0.5, 0.5]\n"
             "      high_light_rate: 1.0\n      high_light_angle: 1.0\nworld_objects:\n" + PLANE)
    with tempfile.TemporaryDirectory() as d:
        w, c = os.path.join(d, "w.yml"), os.path.join(d, "c.yml")
        with open(w, "w") as f:
            f.write(world)
        with open(c, "w") as f:
            f.write(camera_yaml(cam_cfg["position"], cam_cfg["front"], cam_cfg["width"], cam_cfg["height"]))
        wo, cam = rt_ref.load_scene(w, c)
    x, y = raise_search.PIXEL
    ray = cam.lens_func(x, y, 0)
    obj, inter, direction, delta, data = wo.intersect(ray)
    assert obj is not None, "the pixel's ray misses the plane"
    t = inter + delta
    return (t.x, t.y, t.z)
