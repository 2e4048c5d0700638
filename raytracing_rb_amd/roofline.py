"""Algorithmic work model of the hot path, frozen.

The path has no dense contraction (no MFMA) and almost no HBM traffic: the
binding roof is FP64 vector arithmetic.  "Algorithmic" work is what the
reference algorithm does — brute force over every object for every ray and,
per shaded hit and light, every object's cover_area — independent of the
exact culls the kernel uses to skip provably-nil tests.  The per-event counts
come from the device itself (``rtx_count_work``, exact and deterministic under
the counter RNG); the FP64-op cost per event is this frozen table (divisions,
square roots and transcendentals count 1 op each):

  Sphere#intersect, miss .................. 24     (sphere.rb:60-75)
  Sphere#intersect, extra on a hit ........ 30     (sphere.rb:76-85)
  Plane#intersect ......................... 20     (plane.rb:38-51)
  Box#intersect ........................... 270    (6 x 45, box.rb:79-97)
  Sphere#cover_area ....................... 24+40  (shadow test + penumbra setup, sphere.rb:28-57)
  Plane/Box#cover_area .................... 20 / 270
  shading + children per hit .............. 120    (ray_tracer.rb:80-158)

FP64 peak of MI355X: 78.6 TFLOP/s dense (vector and matrix FP64 are the same
rate on CDNA4; 256 CU x 2.4 GHz x 128 FLOP/clk).  HBM peak: 8.0 TB/s.
"""

COST = {
    "sphere_tests": 24,
    "sphere_hits": 30,
    "plane_tests": 20,
    "box_tests": 270,
    "cover_sphere": 24 + 40,
    "cover_plane": 20,
    "cover_box": 270,
    "shade_hits": 120,
}
FP64_PEAK_TFLOPS = 78.6
HBM_PEAK_GBS = 8000.0
FRAMEBUFFER_BYTES_PER_PX = 24      # float64 RGB written once per pixel


def algorithmic_ops(counts):
    return sum(COST[k] * int(counts.get(k, 0)) for k in COST)
