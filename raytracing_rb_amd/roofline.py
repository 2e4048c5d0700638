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

# The dominant (ray-tree) kernel of each engine, as rocprofv3 names it (the
# bounce levels run k_level_c when the hit rings fit LDS, else k_level).
DOMINANT_KERNEL = {"lanes": "k_render", "levels": ("k_level_c", "k_level")}

# FP64 FLOP per lane of one wave instruction of each counted class.
F64_FLOP = {"SQ_INSTS_VALU_FMA_F64": 2, "SQ_INSTS_VALU_ADD_F64": 1, "SQ_INSTS_VALU_MUL_F64": 1,
            "SQ_INSTS_VALU_TRANS_F64": 1}


def kernel_source_sha():
    """Identity of the kernel build: sha256 over the device sources and build flags
    (the value librtx.so embeds, rtx_build_id)."""
    from . import _build
    return _build.source_sha()


def active_lanes(per_frame):
    """Mean active lanes of the VALU: rocprofv3's own VALUUtilization expression on
    gfx950 (profiles/gfx950_counters.txt) is 100 * SQ_THREAD_CYCLES_VALU /
    (SQ_ACTIVE_INST_VALU * 64), so the lanes are THREAD_CYCLES / ACTIVE_INST_VALU.
    Without SQ_ACTIVE_INST_VALU: THREAD_CYCLES / SQ_INSTS_VALU (one issue cycle per
    instruction)."""
    tc = per_frame.get("SQ_THREAD_CYCLES_VALU")
    ac = per_frame.get("SQ_ACTIVE_INST_VALU")
    ni = per_frame.get("SQ_INSTS_VALU")
    if tc and ac:
        return min(64.0, tc / ac), "SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU (rocprofv3 VALUUtilization)"
    if tc and ni:
        return min(64.0, tc / ni), "SQ_THREAD_CYCLES_VALU / SQ_INSTS_VALU"
    return None, None


def hw_fp64(pm, kernel_ms_per_frame):
    """Hardware FP64 rate of the dominant kernel from a PMC profile (tools/pmc_json.py)."""
    pf = pm.get("per_frame") or {}
    if not all(k in pf for k in F64_FLOP):
        return None
    lanes, how = active_lanes(pf)
    if lanes is None:
        return None
    wave_flop = sum(F64_FLOP[k] * pf[k] for k in F64_FLOP)      # FP64 FLOP per lane, summed over waves
    flop = wave_flop * lanes
    ach = flop / (kernel_ms_per_frame * 1e-3) / 1e12
    direct = None
    if "SQ_INSTS_VALU_FLOPS_FP64" in pf:
        # The SQ's own FP64 FLOP counter sums FLOP per lane over wave
        # instructions (measured: it equals 2 FMA + ADD + MUL of the class
        # counters, profiles/r02e), i.e. it is not lane-weighted either: the
        # cross-check of `wave_flop`.
        df = pf["SQ_INSTS_VALU_FLOPS_FP64"] + pf.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0.0)
        direct = {"wave_flop_per_frame": df, "class_wave_flop_per_frame": wave_flop,
                  "fp64_flop_per_frame": df * lanes,
                  "achieved_tflops": round(df * lanes / (kernel_ms_per_frame * 1e-3) / 1e12, 4),
                  "from": "(SQ_INSTS_VALU_FLOPS_FP64 + SQ_INSTS_VALU_FLOPS_FP64_TRANS) x mean active lanes"}
    return {"achieved_tflops": round(ach, 4), "frac": round(ach / FP64_PEAK_TFLOPS, 5), "direct_counter": direct,
            "method": "sum over FP64 VALU classes of FLOP/lane (FMA 2, ADD/MUL/TRANS 1) x wave instructions "
                      "x mean active lanes",
            "fp64_flop_per_frame": flop, "f64_wave_instrs_per_frame": {k: pf[k] for k in F64_FLOP},
            "active_lanes": round(lanes, 2), "active_lanes_from": how,
            "valu_wave_instrs_per_frame": pf.get("SQ_INSTS_VALU"),
            "f64_share_of_valu": round(sum(pf[k] for k in F64_FLOP) / pf["SQ_INSTS_VALU"], 4)
            if pf.get("SQ_INSTS_VALU") else None,
            "valu_busy": valu_busy(pm)}


def valu_busy(pm):
    """rocprofv3's VALUBusy for the dominant kernel (profiles/gfx950_counters.txt:
    100 * SQ_ACTIVE_INST_VALU / CU_NUM / GRBM_GUI_ACTIVE): the share of the
    CUs' active cycles in which the vector ALU issues.  The issue-rate view of
    the same kernel beside the FP64 FLOP rate (an FP64 FMA, an FP32 compare
    and an integer add each occupy an issue slot).

    rocprofv3 on gfx950 reports GRBM_GUI_ACTIVE as the sum over the 8 XCDs'
    clocks (MI355X_MICROARCH.md, DVFS note: effective clock = GRBM_GUI_ACTIVE / 8
    / wall time), and the counter_defs.yaml expression, written for one graphics
    engine, divides by that sum: its figure is 8x low.  `percent` divides by one
    XCD's clock; `rocprof_formula` keeps the literal expression's value."""
    pf = pm.get("per_frame") or {}
    cus = pm.get("cu_num") or 256
    xcds = pm.get("xcd_num") or 8
    if not pf.get("GRBM_GUI_ACTIVE") or not pf.get("SQ_ACTIVE_INST_VALU"):
        return None
    lit = 100.0 * pf["SQ_ACTIVE_INST_VALU"] / cus / pf["GRBM_GUI_ACTIVE"]
    return {"percent": round(lit * xcds, 2), "rocprof_formula": round(lit, 2),
            "from": "100 * SQ_ACTIVE_INST_VALU / CU_NUM / (GRBM_GUI_ACTIVE / %d XCDs), per frame "
                    "(rocprofv3 VALUBusy with GRBM_GUI_ACTIVE taken per XCD)" % xcds}
