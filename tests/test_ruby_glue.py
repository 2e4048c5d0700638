"""The Ruby binding (ext/rtx/lib/rtx.rb, Fiddle) stays in sync with the C-ABI
(include/rtx.h): every struct's field list (names, C types, array sizes, order)
and every exported function's signature are parsed from both files and
compared.  No Ruby interpreter is in this image, so the glue itself cannot run
here; this is what can be checked without one (CPU test)."""

import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "rtx.h")
RUBY = os.path.join(ROOT, "ext", "rtx", "lib", "rtx.rb")
GLUE = os.path.join(ROOT, "ext", "rtx", "lib", "rtx", "reference.rb")

# The Vec3 functions take and return rtx_vec3 by value (not bindable through
# Fiddle::Importer); rtx.rb says so and the glue does not need them.
UNBOUND = re.compile(r"^rtx_vec3_")


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _c_type(decl):
    """A C declaration (type + optional name, optional [n]) -> the Fiddle type string."""
    decl = decl.strip()
    ptr = "*" in decl or "[" in decl
    words = [w for w in re.sub(r"[\*\[\]]|\bconst\b", " ", decl).split() if not re.fullmatch(r"\d+|RTX_\w+", w)]
    base = words[0]
    if ptr:
        return "char*" if base == "char" else "void*"
    return {"rtx_status": "int", "int32_t": "int", "int": "int", "uint64_t": "unsigned long long",
            "int64_t": "long long", "size_t": "size_t", "double": "double", "void": "void",
            "rtx_vec3": "rtx_vec3"}[base]


def header_functions():
    s = " ".join(_strip_c_comments(open(HEADER).read()).split())
    out = {}
    for m in re.finditer(r"((?:const\s+)?\w+\s*\**)\s*\b(rtx_\w+)\s*\(([^()]*)\)\s*;", s):
        ret, name, params = m.group(1), m.group(2), m.group(3).strip()
        args = [] if params in ("", "void") else [_c_type(p) for p in params.split(",")]
        out[name] = (_c_type(ret), tuple(args))
    return out


def header_structs():
    s = _strip_c_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"typedef struct (\w+) \{(.*?)\} \1;", s, flags=re.S):
        fields = []
        for line in m.group(2).split(";"):
            line = " ".join(line.split())
            if not line:
                continue
            first, *rest = line.split(",")
            mm = re.match(r"(.*?)(\**)\s*(\w+)(\[\d+\])?$", first.strip())
            base = (mm.group(1) + mm.group(2)).strip()
            names = [(mm.group(3), mm.group(4) or "")] + [
                (re.match(r"\s*(\w+)(\[\d+\])?", r).group(1), re.match(r"\s*(\w+)(\[\d+\])?", r).group(2) or "")
                for r in rest]
            for n, arr in names:
                fields.append((_c_type(base), n + arr))
        out[m.group(1)] = fields
    return out


def ruby_functions():
    out = {}
    for m in re.finditer(r"^\s*extern '([^']*)'", open(RUBY).read(), flags=re.M):
        mm = re.match(r"(.*?)\s*\b(rtx_\w+)\((.*)\)$", m.group(1))
        params = mm.group(3).strip()
        out[mm.group(2)] = (mm.group(1).strip(), tuple(p.strip() for p in params.split(",")) if params else ())
    return out


def ruby_structs():
    src = open(RUBY).read()
    out = {}
    for m in re.finditer(r"(\w+) = struct \[(.*?)\]\n", src, flags=re.S):
        fields = []
        for f in re.findall(r"'([^']*)'", m.group(2)):
            mm = re.match(r"(.*?)\s*(\w+(\[\d+\])?)$", f)
            fields.append((mm.group(1).strip(), mm.group(2)))
        out[m.group(1)] = fields
    return out


RUBY_STRUCT = {"ObjectDesc": "rtx_object_desc", "LightDesc": "rtx_light_desc", "TextureDesc": "rtx_texture_desc",
               "SceneDesc": "rtx_scene_desc", "CameraDesc": "rtx_camera_desc"}


def test_header_parse_sanity():
    fns = header_functions()
    assert fns["rtx_render"] == ("int", ("void*", "int", "int", "int", "int", "unsigned long long", "void*", "size_t"))
    assert fns["rtx_set_option"] == ("int", ("void*", "char*", "long long"))
    assert fns["rtx_last_error"][0] == "char*"
    assert fns["rtx_rand"][0] == "double"
    st = header_structs()
    assert ("double", "u_unit") in st["rtx_object_desc"] and ("double", "v_unit") in st["rtx_object_desc"]
    assert st["rtx_texture_desc"] == [("int", "width"), ("int", "height"), ("void*", "rgb")]


def test_ruby_structs_match_header():
    h, r = header_structs(), ruby_structs()
    for rb, c in RUBY_STRUCT.items():
        assert r[rb] == h[c], (rb, [x for x in zip(r[rb], h[c]) if x[0] != x[1]][:3])
    # every descriptor struct the header passes across the boundary is bound
    assert set(RUBY_STRUCT.values()) == set(h) - {"rtx_vec3"}


@pytest.mark.parametrize("name", sorted(n for n in header_functions() if not UNBOUND.match(n)))
def test_ruby_extern_matches_header(name):
    r = ruby_functions()
    assert name in r, "include/rtx.h exports %s but ext/rtx/lib/rtx.rb does not bind it" % name
    assert r[name] == header_functions()[name], name


def test_ruby_binds_nothing_the_header_lacks():
    extra = set(ruby_functions()) - set(header_functions())
    assert not extra, extra


def test_glue_replaces_the_reference_call_sites():
    """The glue prepends to the reference classes and overrides exactly the
    hot-path methods (camera.rb:41-110, ray_tracer.rb:16-46,181-195)."""
    g = open(GLUE).read()
    for cls in ("Alex::World.prepend", "Alex::Camera.prepend", "Alex::RayTracer.prepend"):
        assert cls in g
    for m in ("render_at", "render_sync", "render_fork", "trace_sync", "path_trace_sync", "rtx_scene_desc"):
        assert re.search(r"^\s*def %s\b" % m, g, flags=re.M), m
    used = set(re.findall(r"RTX\.(rtx_\w+)\(", g))
    assert used <= set(ruby_functions()), used - set(ruby_functions())
    ref = "/root/reference/src/camera.rb"
    if os.path.exists(ref):       # the methods the glue overrides exist in the reference
        cam = open(ref).read()
        for m in ("render_at", "render_sync", "render_fork"):
            assert re.search(r"def %s\(" % m, cam), m
