#!/usr/bin/env python3
"""Generate the committed golden fixtures from the pure-Python restatement
(oracle/rt_ref.py — a line-by-line restatement of the Ruby reference; the
reference itself cannot run here: no Ruby interpreter).

Fixtures (numpy .npz, data only):
  frame_<name>.npz  float64 framebuffer [H, W, 3] + per-pixel raise status for a
                    committed scene at a reduced size (scene YAML sha256 kept to
                    detect drift)
  vectors.npz       counter-RNG values, Camera#lens_func rays, trace_sync colours
  c2_full_columns64.npz  every 64th column of the full-size C2 frame, by the C
                    restatement (the GPU test renders the whole frame)
  c4_full_columns256.npz every 256th column of the full-size C4 frame (3840x2160,
                    8xAA, depth 8, 4096 spheres), by the C restatement
  frame_c4_48x27.npz the 4096-sphere C4 scene: rendered by the C restatement
                    (oracle/rt_oracle.c, bit-checked against rt_ref.py on the other
                    frames and on sampled C4 pixels in tests/test_oracle.py), since
                    the pure-Python walk over 4097 objects would take hours

    python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import rt_ref  # noqa: E402
from oracle.rb_vec3 import RtxError  # noqa: E402
from oracle.rng import rtx_rand  # noqa: E402

SC = os.path.join(ROOT, "scenes")

# name -> (world, camera, overrides)
FRAMES = {
    "c1_64x36": ("c1_world.yml", "c1_camera.yml", {"width": 64, "height": 36}),
    "c0_48x27": ("c0_world.yml", "camera.yml", {"width": 48, "height": 27}),      # pre 3 / max 10: adaptive
    "c2_32x18": ("c2_world.yml", "c2_camera.yml", {"width": 32, "height": 18}),
    "mix_24x14": ("mix_world.yml", "mix_camera.yml", {"width": 24, "height": 14}),
}


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def render(world, camera, ov, seed=1):
    w, cam = rt_ref.load_scene(os.path.join(SC, world), os.path.join(SC, camera), seed=seed, overrides=ov)
    W, H = cam.width, cam.height
    fb = np.zeros((H, W, 3), np.float64)
    st = np.zeros((H, W), np.int32)
    codes = {"zero_vec": 1, "color_gt1": 2, "domain": 3}
    for x in range(W):
        for y in range(H):
            try:
                fb[y, x] = cam.render_at(x, y).to_a()
            except RtxError as e:
                st[y, x] = codes[e.kind]
    return fb, st


def vectors():
    rs = np.random.RandomState(5)
    keys = np.stack([rs.randint(0, 4000, 300), rs.randint(0, 3000, 300), rs.randint(0, 16, 300),
                     rs.randint(0, 2 ** 31, 300).astype(np.int64) * 977, rs.randint(0, 8, 300)], 1)
    rng = np.array([rtx_rand(1, int(k[0]), int(k[1]), int(k[2]), int(k[3]), int(k[4])) for k in keys])
    w, cam = rt_ref.load_scene(os.path.join(SC, "c2_world.yml"), os.path.join(SC, "c2_camera.yml"), seed=1)
    pix = np.stack([rs.randint(0, 1920, 64), rs.randint(0, 1080, 64), rs.randint(0, 4, 64)], 1).astype(np.int32)
    lens = []
    for x, y, j in pix:
        r = cam.lens_func(int(x), int(y), int(j))
        lens.append(r.front.to_a() + r.position.to_a())
    lens = np.array(lens)
    trace = np.array([cam.ray_tracer.trace_sync(int(x), int(y), cam.lens_func(int(x), int(y), int(j)),
                                                int(j)).to_a() for x, y, j in pix])
    return dict(rng_keys=keys, rng=rng, lens_keys=pix, lens=lens, trace=trace,
                scene_sha=sha(os.path.join(SC, "c2_world.yml")))


C_FRAMES = {
    "c4_48x27": ("c4_world.yml", "c4_camera.yml", {"width": 48, "height": 27}),
}


def render_c(world, camera, ov, seed=1):
    from oracle.c_oracle import Oracle
    from raytracing_rb_amd import config
    sd, cd = config.load_scene(os.path.join(SC, world), os.path.join(SC, camera), camera_overrides=ov)
    fb, st, rc = Oracle(sd, cd).render(seed=seed)
    return fb, st.astype(np.int32)


def c2_columns(stride=64, nprocs=8):
    """C2 (the metric config) at its full 1920x1080, 4xAA, depth 5: every
    `stride`-th column (30 columns, 32,400 pixels) by the C restatement in
    forked column bands (oracle/rt_oracle.c rto_render_fork)."""
    from oracle.c_oracle import Oracle
    from raytracing_rb_amd import config
    sd, cd = config.load_scene(os.path.join(SC, "c2_world.yml"), os.path.join(SC, "c2_camera.yml"))
    full = Oracle(sd, cd).render_fork(nprocs, stride)
    cols = np.arange(0, cd.width, stride)
    np.savez_compressed(os.path.join(HERE, "c2_full_columns%d.npz" % stride), columns=cols,
                        frame=full[:, cols, :], scene_sha=sha(os.path.join(SC, "c2_world.yml")),
                        camera_sha=sha(os.path.join(SC, "c2_camera.yml")), seed=1, source="rt_oracle.c")
    print("c2 columns", cols.size, full[:, cols].mean(axis=(0, 1)))


def c4_columns(stride=256, nprocs=8):
    """C4 (the LDS scene-staging stress config) at its full 3840x2160, 8xAA,
    depth 8 over 4,097 objects: every `stride`-th column (15 columns, 32,400
    pixels) by the C restatement in forked column bands (rto_render_fork, the
    fork_jobs counterpart, camera.rb:41-68).  The world file is generated
    (tools/make_scenes.py ensure_c4, seeded), so its sha is kept to detect drift."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_scenes
    from oracle.c_oracle import Oracle
    from raytracing_rb_amd import config
    world = make_scenes.ensure_c4()
    sd, cd = config.load_scene(world, os.path.join(SC, "c4_camera.yml"))
    full = Oracle(sd, cd).render_fork(nprocs, stride)
    cols = np.arange(0, cd.width, stride)
    np.savez_compressed(os.path.join(HERE, "c4_full_columns%d.npz" % stride), columns=cols,
                        frame=full[:, cols, :], scene_sha=sha(world),
                        camera_sha=sha(os.path.join(SC, "c4_camera.yml")), seed=1, source="rt_oracle.c")
    print("c4 columns", cols.size, full[:, cols].mean(axis=(0, 1)))


def main(only=None):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_scenes
    make_scenes.ensure_c4()
    for name, (world, camera, ov) in C_FRAMES.items():
        if only and name not in only:
            continue
        fb, st = render_c(world, camera, ov)
        np.savez_compressed(os.path.join(HERE, "frame_%s.npz" % name), frame=fb, status=st,
                            world=world, camera=camera, overrides=repr(ov),
                            scene_sha=sha(os.path.join(SC, world)), seed=1, source="rt_oracle.c")
        print(name, fb.shape, "errors", int((st != 0).sum()), "mean", fb.mean(axis=(0, 1)))
    for name, (world, camera, ov) in FRAMES.items():
        if only and name not in only:
            continue
        fb, st = render(world, camera, ov)
        np.savez_compressed(os.path.join(HERE, "frame_%s.npz" % name), frame=fb, status=st,
                            world=world, camera=camera, overrides=repr(ov),
                            scene_sha=sha(os.path.join(SC, world)), seed=1)
        print(name, fb.shape, "errors", int((st != 0).sum()), "mean", fb.mean(axis=(0, 1)))
    if not only or "c2_columns" in only:
        c2_columns()
    if not only or "c4_columns" in only:
        c4_columns()
    if not only or "vectors" in only:
        np.savez_compressed(os.path.join(HERE, "vectors.npz"), **vectors())
        print("vectors")


if __name__ == "__main__":
    main(sys.argv[1:])
