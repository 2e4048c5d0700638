"""Counter-based RNG contract (oracle copy) — TEST INFRASTRUCTURE ONLY.

The reference draws from Ruby's single global MT19937 stream (``Random.rand``,
seeded by ``Random.srand(1)`` at ``src/main.rb:10``) in LIFO ray-processing order:
one draw per camera sample (``src/camera.rb:135``) and two per path-tracing ray
(``src/objects/world_object.rb:84``).  A sequential global stream cannot be
reproduced by independent GPU lanes, so the build replaces it with a keyed hash
(SURVEY.md §7.1):

    u = rtx_rand(seed, x, y, sample, path, draw)  in [0, 1), 53-bit resolution

* lens draw (camera.rb:135):        path = 0,       draw = 0
* path-tracing ray k (world_object.rb:84): path = id of the shaded ray,
                                     draw = 2k (theta, drawn first), 2k+1 (phi)
* ray-path ids: root = 1; child = parent * R + slot with R = pt_times + 3,
  slot 1 = reflection, 2 = refraction, 3 + k = path-tracing ray k (mod 2**64).

Integer-only, so every implementation (this file, ``rt_oracle.c`` and the HIP
kernels) produces identical bits.
"""

MASK64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
OFFSET = 0x632BE59BD9B4E019


def fmix64(h: int) -> int:
    h ^= h >> 33
    h = (h * 0xFF51AFD7ED558CCD) & MASK64
    h ^= h >> 33
    h = (h * 0xC4CEB9FE1A85EC53) & MASK64
    h ^= h >> 33
    return h


def rtx_rand(seed: int, x: int, y: int, sample: int, path: int, draw: int) -> float:
    h = (seed * GOLDEN + OFFSET) & MASK64
    h = fmix64(h ^ (((x & 0xFFFFFFFF) << 32) | (y & 0xFFFFFFFF)))
    h = fmix64(h ^ (((sample & 0xFFFFFFFF) << 32) | (draw & 0xFFFFFFFF)))
    h = fmix64(h ^ (path & MASK64))
    return (h >> 11) * (1.0 / 9007199254740992.0)


def child_path(parent: int, slot: int, pt_times: int) -> int:
    return (parent * (pt_times + 3) + slot) & MASK64
