"""Parity on seeded random scenes (tests/fuzz_scenes.py), through the C-ABI:
every object kind and material path, 1-3 point / area lights, random sampling
(pre / max samples, variance threshold), depth 1-6 and path tracing.  The
default engine against the C oracle (RMS <= 1e-4 per channel, the north-star
tolerance; max |diff| <= 1e-6: only sin/cos/asin/acos round differently,
DESIGN.md §2), the same reference raise at the same pixel, and the engines /
walks against each other bit for bit."""

import re

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_scene_matches_oracle(gpu, tmp_path, seed):
    import fuzz_scenes
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import Renderer, RtxError
    from oracle.c_oracle import Oracle
    w, c = fuzz_scenes.make(seed, tmp_path, 48, 27)
    sd, cd = config.load_scene(w, c)
    ref, st, rc = Oracle(sd, cd).render(seed=seed)
    frames = {}
    for name, opts in (("levels", {}), ("lanes", {"engine": 0}), ("linear", {"bvh": 0}), ("hier", {"bvh": 2})):
        r = Renderer(sd, cd, device=0)
        for k, v in opts.items():
            r.set_option(k, v)
        if rc:
            # the first raise in render_sync order, as the oracle's
            with pytest.raises(RtxError) as e:
                r.render(seed=seed)
            m = re.search(r"pixel \((\d+),(\d+)\)", str(e.value))
            x, y = int(m.group(1)), int(m.group(2))
            first = min((x_ * cd.height + y_ for y_, x_ in zip(*np.nonzero(st))))
            assert (x, y) == (first // cd.height, first % cd.height), (name, str(e.value))
            assert e.value.status == rc, (name, str(e.value))
        else:
            frames[name] = r.render(seed=seed)
        r.close()
    if rc:
        return
    fb = frames["levels"]
    d = fb - ref
    rms = np.sqrt((d.reshape(-1, 3) ** 2).mean(axis=0))
    assert (rms <= 1e-4).all(), rms
    assert np.abs(d).max() <= 1e-6, np.abs(d).max()
    for name in ("lanes", "linear", "hier"):
        assert np.array_equal(frames[name].view(np.uint64), fb.view(np.uint64)), name
