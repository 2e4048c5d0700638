"""CPU oracle for the rtx hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import, call, link or execute anything in this directory, and only as the
*checker* (never as the thing measured or shipped).  The product path
(``raytracing_rb_amd``) never imports this package and fails loudly when its HIP
library is missing.

Contents
--------
* ``rb_vec3.py``  — restatement of the reference's only native code, the boxed
  ``Fast4DMatrix::Vec3`` (``ext/fast_4d_matrix/fast_4d_matrix.c:57-305``).
* ``rng.py``      — the counter-based RNG contract that replaces Ruby's global
  ``Random.rand`` stream.
* ``rt_ref.py``   — pure-Python, line-by-line restatement of the reference's hot
  path (``src/camera.rb``, ``src/ray_tracer.rb``, ``src/world.rb``,
  ``src/objects/*.rb``, ``src/configurable_object.rb``) — slow; small images only.
* ``rt_oracle.c`` — the same semantics restated in plain C (gcc, FP64,
  ``-ffp-contract=off``, glibc libm) — fast; checked bit-for-bit against
  ``rt_ref.py``; also the fork()-per-core CPU baseline (``src/fork_jobs.rb``).

Pinning
-------
* The Vec3 layer is pinned by the reference's own known-answer tests
  (``spec/fast_4d_matrix_spec.rb:6-113``), see ``tests/test_vec3_spec.py``.
* The ray-tracing layers have NO runnable reference here (no Ruby interpreter,
  no ``ruby.h``, no gems) and no golden images in the reference:
  **parity unpinned** against a live reference for rendering.  They are pinned
  by two independent restatements (``rt_ref.py`` and ``rt_oracle.c``) that must
  agree bit for bit, and by committed golden fixtures generated from
  ``rt_ref.py`` (``tests/golden/make_golden.py``).
"""
