"""Build librtx.so in-tree with hipcc for gfx950 (no JIT cache, no pip install).

    python -m raytracing_rb_amd._build [--force]
"""

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "librtx.so")
SOURCES = [os.path.join(CSRC, f) for f in ("rtx_kernels.hip", "rtx_levels.hip", "rtx_capi.cpp")]
HEADERS = [os.path.join(CSRC, f) for f in ("rtx_scene.h", "rtx_vec3.h", "rtx_launch.h", "rtx_device.h", "rtx_bvh_build.h")] + [
    os.path.join(ROOT, "include", "rtx.h")]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off: no FMA contraction anywhere — every binary64 operation rounds
# exactly like the reference's Ruby + C-extension arithmetic.
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-ffp-contract=off", "-fno-fast-math", "-std=c++17", "-fPIC",
         "-Wall", "-Wno-unused-result", "-Wno-unused-value"]


# RCCL for rtx_render_multi's gather over xGMI (librccl.so ships with ROCm).
LIBS = ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]


CLI_SRC = os.path.join(HERE, "cli", "rtx_main.cpp")
CLI_DEPS = [CLI_SRC] + [os.path.join(HERE, "cli", f) for f in ("yaml_lite.hpp", "png_io.hpp", "scene_load.hpp")] + [
    os.path.join(ROOT, "include", "rtx.h")]
CLI_OUT = os.path.join(HERE, "rtx")


def build_cli(force=False, verbose=False):
    """The native CLI (counterpart of src/main.rb): g++ over librtx.so + zlib."""
    if not force and os.path.exists(CLI_OUT) and all(
            os.path.getmtime(p) <= os.path.getmtime(CLI_OUT) for p in CLI_DEPS + [OUT]):
        return CLI_OUT
    tmp = "%s.%d.tmp" % (CLI_OUT, os.getpid())   # (parallel test workers may rebuild it at once)
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-o", tmp, CLI_SRC, "-L" + HERE, "-l:librtx.so",
           "-lz", "-lpthread", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, CLI_OUT)
    return CLI_OUT


def source_sha(extra=()):
    """Identity of the kernel build: sha256 over the device sources, headers and
    build flags, plus any extra defines (embedded in librtx.so as rtx_build_id,
    checked at load against the no-defines identity: a diagnostic build written
    in place of the production library is refused)."""
    import hashlib
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS).encode())
    if extra:
        h.update(("\0" + " ".join(extra)).encode())
    return h.hexdigest()[:16]


def stale():
    if not os.path.exists(OUT):
        return True
    # a diagnostic build (defines) written over the production library is stale,
    # and so is one whose sources changed while it compiled (the identity it embeds)
    odir = os.path.join(ROOT, "build", "obj", os.path.basename(OUT))
    tag, ident = os.path.join(odir, "flags"), os.path.join(odir, "built_sha")
    if not os.path.exists(tag) or open(tag).read() != " ".join(FLAGS):
        return True
    if not os.path.exists(ident) or open(ident).read() != source_sha():
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in SOURCES + HEADERS + [__file__])


def build(force=False, verbose=False, out=None, defines=()):
    """Each translation unit compiled to an object in parallel (build/obj/), then linked."""
    out = out or OUT
    if not force and out == OUT and not stale():
        return OUT
    # `defines`: NAME[=VALUE] macros; entries starting with "-" are raw compiler flags
    dflags = [d if d.startswith("-") else "-D" + d for d in defines]
    odir = os.path.join(ROOT, "build", "obj", os.path.basename(out))
    os.makedirs(odir, exist_ok=True)
    objs, procs = [], []
    tag = os.path.join(odir, "flags")                # objects are reused only under the same flags
    same = os.path.exists(tag) and open(tag).read() == " ".join(FLAGS + dflags)
    with open(tag, "w") as f:
        f.write(" ".join(FLAGS + dflags))
    newest_dep = max(os.path.getmtime(p) for p in HEADERS + [__file__])
    sha = source_sha(dflags)
    for src in SOURCES:
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        objs.append(obj)
        ident = []
        if src.endswith("rtx_capi.cpp"):          # the build identity, always current (a quick unit)
            ident = ['-DRTX_SOURCE_SHA="%s"' % sha]
        elif same and os.path.exists(obj) and os.path.getmtime(obj) > max(newest_dep, os.path.getmtime(src)):
            continue
        cmd = [HIPCC] + FLAGS + dflags + ident + ["-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), cmd))
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", out + ".tmp"] + objs + LIBS
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    with open(os.path.join(odir, "built_sha"), "w") as f:
        f.write(sha)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    build_cli(force="--force" in sys.argv, verbose=True)
