"""Every tuning option librtx accepts (rtx_get_option's table in rtx_capi.cpp)
is documented in include/rtx.h's option list, with its default."""

import os
import re

from conftest import ROOT


def _options():
    src = open(os.path.join(ROOT, "raytracing_rb_amd", "csrc", "rtx_capi.cpp")).read()
    tab = src[src.index("const struct { const char* k; int64_t v; } tab[] = {"):]
    tab = tab[:tab.index("};")]
    return re.findall(r'\{"(\w+)", c->opt_\w+\}', tab)


def test_every_option_is_documented_in_the_header():
    names = _options()
    assert len(names) >= 20 and "lv_sort" in names and "exact_raises" in names
    hdr = open(os.path.join(ROOT, "include", "rtx.h")).read()
    missing = [n for n in names if '"%s"' % n not in hdr]
    assert not missing, missing


def test_every_option_setter_validates_its_key():
    src = open(os.path.join(ROOT, "raytracing_rb_amd", "csrc", "rtx_capi.cpp")).read()
    setter = src[src.index("rtx_status rtx_set_option("):]
    for n in _options():
        assert '"%s"' % n in setter, n
