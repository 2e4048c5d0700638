"""Regenerate tests/golden/raise_scenes.json (test infrastructure):
tools/raise_search.py's configurations, the pixel cases' T from the Python
restatement (tests/raise_cases.py).   python tests/golden/make_raise_scenes.py"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))
import raise_cases  # noqa: E402

res = raise_cases.raise_search.search_all(raise_cases.pixel_T())
with open(os.path.join(HERE, "raise_scenes.json"), "w") as f:
    json.dump(res, f, indent=1)
    f.write("\n")
print(json.dumps({k: v["tries"] for k, v in res.items()}))
