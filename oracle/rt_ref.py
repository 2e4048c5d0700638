"""Pure-Python restatement of the reference hot path — TEST INFRASTRUCTURE ONLY.

A line-by-line restatement of the Ruby semantics, written for review against the
Ruby files it cites.  Slow (pure-Python loops): use it on small images only.  It
is the generator of the committed golden fixtures (``tests/golden/``) and the
bit-exact cross-check of the C oracle (``rt_oracle.c``).

Deliberate, documented departures from the Ruby program:
* ``Random.rand`` is replaced by the counter RNG of ``oracle/rng.py``.
* ``World#high_lights`` evaluates ``lit_area`` only for its truthiness, which is
  always true in Ruby (``world.rb:92-93``); it is evaluated here (and in the C
  oracle, and on the GPU) because its ``Sphere#cover_area`` can raise.
* The ``LOG.logt`` trace (``logger.rb``) is not emitted (no effect on pixels).
* Texture files are decoded by Pillow (``>>8`` on 16-bit samples, matching
  RMagick's ``(pixel.red >> 8)`` at ``texture.rb:19``).
"""

import math
import os

from .rb_vec3 import RtxError, Vec3
from .rng import child_path, rtx_rand

EPSILON = 1e-5                     # src/libs/algebra.rb:2


class Ray:                         # src/libs/algebra.rb:3-17
    __slots__ = ("front", "position")

    def __init__(self, front, position):
        self.front = front
        self.position = position

    def distance(self, pos):
        return (self.position - pos).r


def _to_i(f):
    """Ruby Float#to_i: truncation; NaN/Inf raise FloatDomainError."""
    if f != f or f in (math.inf, -math.inf):
        raise RtxError("domain", "FloatDomainError: %r" % f)
    return int(f)


def _acos(x):
    try:
        return math.acos(x)
    except ValueError:
        raise RtxError("domain", "Math::DomainError acos(%r)" % x)


def _asin(x):
    try:
        return math.asin(x)
    except ValueError:
        raise RtxError("domain", "Math::DomainError asin(%r)" % x)


def _sqrt(x):
    try:
        return math.sqrt(x)
    except ValueError:
        raise RtxError("domain", "Math::DomainError sqrt(%r)" % x)


# ---------------------------------------------------------------- textures
class Texture:
    """src/objects/texture.rb:8-28; ``rows`` = decoded 8-bit RGB rows, top-down."""

    def __init__(self, rows, horizontal_scale, vertical_scale, u_off=None, v_off=None):
        self.h_scale = horizontal_scale
        self.v_scale = vertical_scale
        self.height = len(rows)
        self.width = len(rows[0])
        self.u_off = 0.0 if u_off is None else u_off
        self.v_off = 0.0 if v_off is None else v_off
        self.data = [[Vec3(r / 256.0, g / 256.0, b / 256.0) for (r, g, b) in row] for row in rows]

    def color(self, uu, vv):
        u = _to_i((uu + self.u_off) / self.h_scale) % self.width     # Ruby % = floor-mod
        v = _to_i((vv + self.v_off) / self.v_scale) % self.height
        return self.data[v][u]


def load_texture_rows(path):
    import numpy as np
    from PIL import Image
    a = np.asarray(Image.open(path).convert("RGB"))
    return [[tuple(int(c) for c in px) for px in row] for row in a]


# ---------------------------------------------------------------- objects
class WorldObject:                 # src/objects/world_object.rb
    reflective_attenuation = None
    refractive_attenuation = None
    refractive_rate = None
    diffuse_rate = None
    ambient = None
    texture = None
    name = None

    def __init__(self, props):
        for k, v in props.items():
            setattr(self, k, v)

    def reflect_refract_vector(self):                 # :33-39
        return self.reflective_attenuation, self.refractive_attenuation

    def cover_area(self, light_position, light_radius, target_position):   # :41-49
        ray = Ray(light_position - target_position, target_position)
        res = self.intersect(ray)
        hit = res[0] if res else None
        if hit is not None and (hit - light_position).dot(target_position - light_position) > 0:
            return 1
        return 0

    def local_lighting(self, position, lights, normal_vector, ray, color_filter=None):  # :51-74
        lc = Vec3(0.0, 0.0, 0.0)
        for light, light_color in lights:
            n = normal_vector.normalize()
            l = (light.position - position).normalize()
            l_dot_n = l.dot(n)
            if l_dot_n > 1:
                l_dot_n = 1.0
            elif l_dot_n < 0:
                l_dot_n = 0.0
            lc = lc + light_color * l_dot_n
        if len(lights) > 0:
            lc = lc / float(len(lights))
        if color_filter is not None:
            return lc * self.diffuse_rate * color_filter + self.ambient
        return lc * self.diffuse_rate + self.ambient

    def path_tracing(self, intersection, n, pt_times, draw):          # :76-90
        ret = []
        att = self.diffuse_rate / float(pt_times)
        for k in range(pt_times):
            front = n.normalize()
            left = _vertical_vector(n).normalize()
            up = front.cross(left)
            theta = draw(2 * k) * math.pi / 2          # theta drawn first
            phi = draw(2 * k + 1) * math.pi * 2
            direction = front * math.sin(theta) + (left * math.cos(phi) + up * math.sin(phi)) * math.cos(theta)
            ret.append((Ray(direction, intersection), att))
        return ret


def _vertical_vector(n):          # world_object.rb:105-120
    if n.r == 0:
        raise RtxError("zero_vec", "zero vector detected")
    a = n.to_a()
    if a[0] == 0:
        if a[1] == 0:
            return Vec3(1.0, 0.0, 0.0)
        return Vec3(0.0, -a[2] / a[1], 1.0)
    return Vec3(-(a[1] + a[2]) / a[0], 1.0, 1.0)


def _reflection(ray, n, intersection, delta):        # world_object.rb:121-125
    cos_theta = ray.front.cos(-n)
    front = (n.normalize() * (2 * cos_theta * ray.front.r) + ray.front).normalize()
    return Ray(front, intersection + delta)


def _refraction(ray, n, intersection, reflection, rate, delta):   # world_object.rb:127-137
    sin_i = _sqrt(1 - ray.front.cos(n) ** 2)
    sin_r = sin_i / rate
    if sin_r >= 1:
        return None
    r = _asin(sin_r)
    direction = n.normalize() * (-math.cos(r)) + (reflection + ray.front).normalize() * sin_r
    return Ray(direction, intersection - n.normalize() * EPSILON)


class Sphere(WorldObject):         # src/objects/sphere.rb
    center = None
    radius = None
    texture_file_path = None

    def __init__(self, props, tex_loader):
        super().__init__(props)
        self.radius = float(self.radius)
        if self.refractive_rate is not None:
            self.refractive_rate = float(self.refractive_rate)
        if self.texture_file_path:
            self.east = self.north_pole_vec.cross(self.greenwich_vec)
            self.texture = Texture(tex_loader(self.texture_file_path),
                                   float(self.texture_horizontal_scale),
                                   float(self.texture_vertical_scale),
                                   _opt_float(getattr(self, "texture_u_offset", None)),
                                   _opt_float(getattr(self, "texture_v_offset", None)))

    def inner(self, position):
        return (position - self.center).r <= self.radius

    def cover_area(self, light_position, light_radius, target_position):    # :28-57
        factor = super().cover_area(light_position, light_radius, target_position)
        lt = light_position - target_position
        t = (self.center - target_position).dot(lt) / lt.r2
        x1 = target_position + lt * t
        r1 = light_radius * ((x1 - target_position).r / lt.r)
        d = (x1 - self.center).r
        R = self.radius
        if d >= r1 + R:
            return 0
        s1 = math.pi * r1 * r1
        if d > abs(R - r1):
            ct1 = min((r1 * r1 + d * d - R * R) / (2 * r1 * d), 1.0)
            ct2 = min((R * R + d * d - r1 * r1) / (2 * R * d), 1.0)
            th1 = _acos(ct1)
            th2 = _acos(ct2)
            ds = ((th1 - math.sin(th1)) * r1 * r1 + (th2 - math.sin(th2)) * R * R) / 2
            return factor * ds / s1
        if r1 > R:
            return factor * math.pi * R * R / s1
        return factor

    def intersect(self, ray):                          # :60-85
        t = (self.center - ray.position).dot(ray.front) / ray.front.r2
        v = ray.front * t
        nearest_point = ray.position + v
        if not self.inner(nearest_point):
            return None
        nearest_dis = (nearest_point - self.center).r
        h = _sqrt(self.radius ** 2 - nearest_dis ** 2)
        vec = ray.front.normalize() * h
        from_inner = self.inner(ray.position)
        direction = "out" if from_inner else "in"
        intersection = nearest_point - vec if direction == "in" else nearest_point + vec
        if not from_inner and t < 0:
            return None
        sign = 1.0 if direction == "in" else -1.0
        return (intersection, direction, (intersection - self.center) * EPSILON * sign, None)

    def intersect_parameters(self, ray, intersection, direction, delta, data=None):   # :88-101
        n = (intersection - self.center) if direction == "in" else (self.center - intersection)
        reflection = _reflection(ray, n, intersection, delta)
        rate = self.refractive_rate if direction == "in" else 1.0 / self.refractive_rate
        refraction = _refraction(ray, n, intersection, reflection.front, rate, delta)
        return n, reflection, refraction

    def get_uv(self, position):                        # :111-120
        vec = position - self.center
        x = vec.dot(self.greenwich_vec.normalize()) / self.radius
        y = vec.dot(self.east.normalize()) / self.radius
        z = vec.dot(self.north_pole_vec.normalize()) / self.radius
        m = _sqrt(x * x + y * y + z * z + 2 * x + 1)
        return (y / m + 1) / 2, (-z / m + 1) / 2

    def local_lighting(self, position, lights, normal_vector, ray, color_filter=None):   # :122-129
        if color_filter is None:
            color_filter = Vec3(1.0, 1.0, 1.0)
        if self.texture is not None:
            u, v = self.get_uv(position)
            return super().local_lighting(position, lights, normal_vector, ray,
                                          self.texture.color(u, v) * color_filter)
        return super().local_lighting(position, lights, normal_vector, ray, color_filter)


class Plane(WorldObject):          # src/objects/plane.rb
    point = None
    front = None
    up = None
    u_unit = None
    v_unit = None
    texture_file_path = None

    def __init__(self, props=None, tex_loader=None):
        if props is None:
            return                                    # Plane.create_from_scratch
        super().__init__(props)
        if self.refractive_rate is not None:
            self.refractive_rate = float(self.refractive_rate)
        if self.texture_file_path:
            self.texture = Texture(tex_loader(self.texture_file_path),
                                   float(self.texture_horizontal_scale),
                                   float(self.texture_vertical_scale))
        self.reinit()

    def reinit(self):                                 # :21-23
        self.left = self.front.cross(self.up).normalize()

    def intersect(self, ray):                         # :38-51
        denominator = self.front.dot(ray.front)
        if denominator == 0:
            return None
        t = (self.point - ray.position).dot(self.front) / denominator
        intersection = ray.position + ray.front * t
        if t < 0:
            return (None, None)
        direction = "in" if self.front.dot(ray.front) < 0 else "out"
        nd = -self.front.dot(ray.front)
        sign = float((nd > 0) - (nd < 0))
        return (intersection, direction, self.front * EPSILON * sign, None)

    def intersect_parameters(self, ray, intersection, direction, delta, data=None):   # :54-67
        n = -self.front if self.front.dot(ray.front) > 0 else self.front
        reflection = _reflection(ray, n, intersection, delta)
        if self.refractive_rate is not None:
            refraction = _refraction(ray, n, intersection, reflection.front, self.refractive_rate, delta)
        else:
            refraction = None
        return n, reflection, refraction

    def get_uv(self, position):                       # :81-85
        u = (position - self.point).dot(self.left.normalize()) / self.u_unit
        v = (position - self.point).dot(self.up.normalize()) / self.v_unit
        return u, v

    def local_lighting(self, position, lights, normal_vector, ray, light_filter=None):   # :87-94
        if light_filter is None:
            light_filter = Vec3(1.0, 1.0, 1.0)
        if self.texture is not None:
            u, v = self.get_uv(position)
            return super().local_lighting(position, lights, normal_vector, ray,
                                          self.texture.color(u, v) * light_filter)
        return super().local_lighting(position, lights, normal_vector, ray, light_filter)


class Box(WorldObject):            # src/objects/box.rb
    point = None
    front = None
    up = None
    width_front = None
    width_up = None
    width_left = None

    def __init__(self, props, tex_loader):
        super().__init__(props)
        wf, wu, wl = float(self.width_front), float(self.width_up), float(self.width_left)
        if self.refractive_rate is not None:
            self.refractive_rate = float(self.refractive_rate)
        left = self.front.cross(self.up).normalize()

        def face(front, up, point, uu, vu):
            p = Plane()
            p.front, p.up, p.point, p.u_unit, p.v_unit = front, up, point, uu, vu
            return p

        self.planes = [
            face(self.up, left, self.point + self.up * wu * 0.5, wf, wl),
            face(-self.up, left, self.point - self.up * wu * 0.5, wf, wl),
            face(self.front, self.up, self.point + self.front * wf * 0.5, wl, wu),
            face(-self.front, self.up, self.point - self.front * wf * 0.5, wl, wu),
            face(left, self.up, self.point + left * wl * 0.5, wf, wu),
            face(-left, self.up, self.point - left * wl * 0.5, wf, wu),
        ]
        for p in self.planes:
            p.reflective_attenuation = self.reflective_attenuation
            p.refractive_attenuation = self.refractive_attenuation
            p.refractive_rate = self.refractive_rate
            p.diffuse_rate = self.diffuse_rate
            p.reinit()

    def intersect(self, ray):                         # :79-97
        nearest_dis = math.inf
        nearest_ret = None
        for index, plane in enumerate(self.planes):
            res = plane.intersect(ray)
            intersection = res[0] if res else None
            if intersection is not None:
                u, v = plane.get_uv(intersection)
                if -0.5 <= u and u <= 0.5 and -0.5 <= v and v <= 0.5:
                    d = (intersection - ray.position).r
                    if d < nearest_dis:
                        nearest_dis = d
                        nearest_ret = (intersection, res[1], res[2], index)
        return nearest_ret

    def intersect_parameters(self, ray, intersection, direction, delta, data=None):   # :100-105
        return self.planes[data].intersect_parameters(ray, intersection, direction, delta)


def _opt_float(v):
    return None if v is None else float(v)


class SpotLight:                   # src/lights/light.rb, spot_light.rb
    def __init__(self, props):
        self.radius = None
        for k, v in props.items():
            setattr(self, k, v)


# ---------------------------------------------------------------- world
class World:                       # src/world.rb
    def __init__(self, cfg, tex_loader):
        self.max_distance = cfg["max_distance"]
        self.soft_shadow_exponent = cfg["soft_shadow_exponent"]
        kinds = {"Sphere": Sphere, "Plane": Plane, "Box": Box}
        self.objects = [kinds[it["type"]](it["properties"], tex_loader) for it in cfg["world_objects"]]
        self.lights = [SpotLight(it["properties"]) for it in cfg["lights"]]

    def intersect(self, ray):                         # :37-59
        nearest = (None, None, None, None, None)
        nearest_dis = self.max_distance
        for obj in self.objects:
            res = obj.intersect(ray)
            if res and res[0] is not None:
                new_dis = ray.distance(res[0])
                if new_dis < nearest_dis:
                    nearest_dis = new_dis
                    nearest = (obj, res[0], res[1], res[2], res[3])
        return nearest

    def lit_area(self, target, light_pos, radius):    # :62-69
        total_area = 1
        for obj in self.objects:
            total_area -= obj.cover_area(light_pos, radius, target)
        return max(total_area, 0)

    def local_lights(self, position):                 # :72-80
        ret = []
        for light in self.lights:
            area = self.lit_area(position, light.position, light.radius)
            if area > 0:
                ret.append((light, light.color * (float(area) ** self.soft_shadow_exponent / len(self.lights))))
        return ret

    def high_lights(self, ray):                       # :83-98
        ret = []
        for light in self.lights:
            a = light.position - ray.position
            cos_theta = ray.front.cos(a)
            if cos_theta < -1:
                cos_theta = -1
            if cos_theta > 1:
                cos_theta = 1
            ang = _acos(cos_theta)
            # `&& lit_area(ray.position, light.position, light.radius, object)`
            # (:92-93): always truthy (a number), but it runs and can raise
            if ang < (light.high_light_angle / 180.0 * math.pi) and \
                    self.lit_area(ray.position, light.position, light.radius) is not None:
                ret.append((light, light.color * float(light.high_light_rate)))
        return ret


# ---------------------------------------------------------------- tracer
class RayTracer:                   # src/ray_tracer.rb
    def __init__(self, world, trace_depth, pt_times, seed):
        self.world = world
        self.trace_depth = trace_depth
        self.pt_times = pt_times
        self.seed = seed

    def trace_sync(self, x, y, ray, sample):          # :16-46
        queue = [(ray, self.trace_depth, Vec3(1.0, 1.0, 1.0), 1)]
        leaves = []
        while queue:
            item = queue.pop()                        # LIFO Array#pop
            rays, lights = self.rt_map(item, x, y, sample)
            leaves.extend(lights)
            queue.extend(rays)
        s = Vec3(0.0, 0.0, 0.0)
        for c in leaves:                              # FIFO Queue drain
            s = self.rt_reduce(s, c)
        return s

    def rt_map(self, item, x, y, sample):             # :50-164
        ray, depth, att, path = item
        children, leaves = [], []
        if depth <= 0 or att.r < 0.0001:
            return children, leaves
        fired = self.world.high_lights(ray)
        for light, color in fired:
            leaves.append(att * color / float(len(fired)))
        if leaves:
            return children, leaves
        obj, intersection, direction, delta, data = self.world.intersect(ray)
        if obj is None:
            return children, leaves
        n, reflection, refraction = obj.intersect_parameters(ray, intersection, direction, delta, data)
        att_reflect, att_refract = obj.reflect_refract_vector()
        pt = self.pt_times
        if reflection is not None:
            children.append((reflection, depth - 1, att * att_reflect, child_path(path, 1, pt)))
        if refraction is not None:
            children.append((refraction, depth - 1, att * att_refract, child_path(path, 2, pt)))
        lights = self.world.local_lights(intersection + delta)
        if len(lights) == 0:
            seed = self.seed
            draw = lambda k: rtx_rand(seed, x, y, sample, path, k)
            for k, (pt_ray, pt_att) in enumerate(obj.path_tracing(intersection + delta, n, pt, draw)):
                children.append((pt_ray, depth - 1, att * pt_att, child_path(path, 3 + k, pt)))
        else:
            leaves.append(att * obj.local_lighting(intersection, lights, n, ray))
        return children, leaves

    def path_trace_sync(self, x, y, ray):             # :181-195 -> path_trace :196-289
        """Dead code in the reference (never called).  Followed to the first
        raise: on any hit, roulette_random (:166-179) sums the
        [action, probability] pairs whose probabilities are never-assigned
        attr_accessors (world_object.rb:12), and `0 + nil` raises TypeError."""
        att = Vec3(1.0, 1.0, 1.0)
        if self.trace_depth <= 0 or att.r < 0.0001:  # :197-201
            return Vec3(0.0, 0.0, 0.0)
        ret = Vec3(0.0, 0.0, 0.0)
        fired = self.world.high_lights(ray)          # :206-214
        for light, color in fired:
            ret = ret + att * color / float(len(fired))
        if fired:
            return ret
        obj, intersection, direction, delta, data = self.world.intersect(ray)   # :217
        if obj is None:                              # :284-288
            return Vec3(0.0, 0.0, 0.0)
        obj.intersect_parameters(ray, intersection, direction, delta, data)    # :219 (may raise first)
        obj.reflect_refract_vector()                 # :224
        raise RtxError("type", "TypeError: nil can't be coerced into Integer")   # :226-229 -> :167

    @staticmethod
    def rt_reduce(c1, c2):                            # :292-298
        ret = c1 + c2
        if not (ret.x <= 1 and ret.y <= 1 and ret.z <= 1):
            raise RtxError("color_gt1", "color greater than 1, %s" % ret.to_s())
        return ret


# ---------------------------------------------------------------- camera
class Camera:                      # src/camera.rb
    def __init__(self, world, cfg, seed=1):
        for k, v in cfg.items():
            setattr(self, k, v)
        self.world = world
        self.seed = seed
        self.ray_tracer = RayTracer(world, self.trace_depth, self.monte_carlo_diffusion_times, seed)

    def lens_func(self, x, y, j):                     # :129-151
        left = self.up.cross(self.front).normalize()
        retina_center = self.position - self.front.normalize() * self.image_distance
        retina_position = (retina_center
                           + left * (2.0 * (x / self.width - 0.5) * self.retina_width)
                           + self.up.normalize() * (2 * (y / self.height - 0.5) * self.retina_height))
        theta = rtx_rand(self.seed, x, y, j, 0, 0)
        rand_vector = (left.normalize() * math.cos(theta) + self.up.normalize() * math.sin(theta)) * self.aperture_radius
        aperture_position = self.position + rand_vector
        object_distance = self.focal_distance * self.image_distance / (self.image_distance - self.focal_distance)
        point_on_focal_plane = self.position + self.front.normalize() * object_distance
        r = Ray(self.position - retina_position, retina_position)
        # intersect_plane (:123-127)
        t = (point_on_focal_plane - r.position).dot(self.front) / self.front.dot(r.front)
        target_point = r.position + r.front * t
        return Ray(target_point - aperture_position, aperture_position)

    def render_at(self, x, y):                        # :70-99
        pre_samples = []
        average = Vec3(0.0, 0.0, 0.0)
        for j in range(self.pre_sample_times):
            v = self.ray_tracer.trace_sync(x, y, self.lens_func(x, y, j), j)
            pre_samples.append(v)
            average = average + v
        variance = 0
        average = average / float(self.pre_sample_times)
        for j in range(self.pre_sample_times):
            variance += max((pre_samples[j] - average).to_a()) ** 2
        variance /= self.pre_sample_times
        if variance >= self.variant_threshold:
            color_vec = Vec3(0.0, 0.0, 0.0)
            for j in range(self.pre_sample_times, self.max_sample_times):
                color_vec = color_vec + self.ray_tracer.trace_sync(x, y, self.lens_func(x, y, j), j)
            average = (average * float(self.pre_sample_times) + color_vec) / float(self.max_sample_times)
        return average

    def render(self, x0=0, y0=0, x1=None, y1=None):
        """Float framebuffer rows y0..y1, cols x0..x1, final orientation (row = y)."""
        x1 = self.width if x1 is None else x1
        y1 = self.height if y1 is None else y1
        out = [[None] * (x1 - x0) for _ in range(y1 - y0)]
        for x in range(x0, x1):                       # render_sync: x outer, y inner
            for y in range(y0, y1):
                out[y - y0][x - x0] = self.render_at(x, y).to_a()
        return out


# ---------------------------------------------------------------- config
def _is_num(v):
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def _parse_vec_hash(h):            # configurable_object.rb:25-41
    out = {}
    for k, v in h.items():
        if isinstance(v, dict):
            out[str(k)] = _parse_vec_hash(v)
        elif isinstance(v, list) and len(v) == 3 and all(_is_num(e) for e in v):
            out[str(k)] = Vec3(*[float(e) for e in v])
        elif isinstance(v, list):
            out[str(k)] = _parse_vec_array(v)
        else:
            out[str(k)] = v
    return out


def _parse_vec_array(a):           # configurable_object.rb:11-23
    out = []
    for v in a:
        if isinstance(v, dict):
            out.append(_parse_vec_hash(v))
        elif isinstance(v, list) and len(v) == 3 and all(_is_num(e) for e in v):
            out.append(Vec3(*[float(e) for e in v]))
        elif isinstance(v, list):
            out.append(_parse_vec_array(v))
    return out


def load_config(path):
    """YAML.load + hash_value_parse_vector (configurable_object.rb:43-49).

    PyYAML (YAML 1.1) needs a '.' in a float; Psych also reads '1e-5' as a
    Float, so that form is added to the resolver."""
    import re
    import yaml

    class _Loader(yaml.SafeLoader):
        pass

    _Loader.add_implicit_resolver(
        "tag:yaml.org,2002:float",
        re.compile(r"^[-+]?(?:[0-9][0-9_]*)(?:\.[0-9_]*)?[eE][-+]?[0-9]+$"),
        list("-+0123456789"))
    with open(path) as f:
        cfg = yaml.load(f, Loader=_Loader)
    return _parse_vec_hash(cfg)


def make_texture_loader(base_dir, remap=None):
    remap = remap or {}

    def loader(p):
        p = remap.get(p, p)
        cand = p if os.path.isabs(p) else os.path.join(base_dir, p)
        if not os.path.exists(cand):
            cand = p
        return load_texture_rows(cand)
    return loader


def load_scene(world_yml, camera_yml, seed=1, overrides=None, remap=None):
    wcfg = load_config(world_yml)
    ccfg = load_config(camera_yml)
    if overrides:
        ccfg.update(overrides)
    world = World(wcfg, make_texture_loader(os.path.dirname(os.path.abspath(world_yml)), remap))
    return world, Camera(world, ccfg, seed)
