"""Independent pure-Python restatement of raytracer.erl's render path.

TEST INFRASTRUCTURE ONLY (oracle/): used by tests/ and the golden-vector
generator to cross-check the C oracle (oracle/rt_oracle.c); never imported by
the product package.  Small cases only (pure-Python loops).

It works on the Erlang terms themselves: records are tuples whose first element
is the record tag (a str, e.g. ``('vector', 4, 0, 10)``), numbers keep their
Erlang int/float type.  Python's int/float arithmetic matches Erlang's for the
operations used here (int op int stays an exact int, mixed operands convert
the int to a double, ``/`` always yields a double) and ``math.sqrt/pow/tan``
wrap the host libm exactly as BEAM's ``math`` BIFs do.  Each function cites
the reference line it restates.
"""
from __future__ import annotations

import math

# record field positions (raytracer.erl:72-81); index 0 is the tag
VX, VY, VZ = 1, 2, 3


def _exact_eq(a, b):
    """Erlang =:= (exact equality: 4 =/= 4.0), used by shadow_factor's match (:263)."""
    if isinstance(a, tuple) or isinstance(b, tuple):
        if not (isinstance(a, tuple) and isinstance(b, tuple)) or len(a) != len(b):
            return False
        return all(_exact_eq(x, y) for x, y in zip(a, b))
    if isinstance(a, list) or isinstance(b, list):
        if not (isinstance(a, list) and isinstance(b, list)) or len(a) != len(b):
            return False
        return all(_exact_eq(x, y) for x, y in zip(a, b))
    if isinstance(a, bool) or isinstance(b, bool):
        return a is b
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return type(a) is type(b) and a == b
    return type(a) is type(b) and a == b


def vec(x, y, z):
    return ('vector', x, y, z)


# ---- vector math, raytracer.erl:524-573 -------------------------------------------
def vector_add(a, b):  # :524-527
    return vec(a[1] + b[1], a[2] + b[2], a[3] + b[3])


def vector_sub(a, b):  # :529-532
    return vec(a[1] - b[1], a[2] - b[2], a[3] - b[3])


def vector_square_mag(v):  # :534-535
    return v[1] * v[1] + v[2] * v[2] + v[3] * v[3]


def vector_mag(v):  # :537-538
    return math.sqrt(vector_square_mag(v))


def vector_scalar_mult(v, s):  # :540-541
    return vec(v[1] * s, v[2] * s, v[3] * s)


def vector_component_mult(a, b):  # :543-544
    return vec(a[1] * b[1], a[2] * b[2], a[3] * b[3])


def vector_dot_product(a, b):  # :546-547
    return a[1] * b[1] + a[2] * b[2] + a[3] * b[3]


def vector_cross_product(a, b):  # :549-552
    a1, a2, a3 = a[1], a[2], a[3]
    b1, b2, b3 = b[1], b[2], b[3]
    return vec(a2 * b3 - a3 * b2, a3 * b1 - a1 * b3, a1 * b2 - a2 * b1)


def vector_normalize(v):  # :554-560
    mag = vector_mag(v)
    if mag == 0:
        return vec(0, 0, 0)
    return vector_scalar_mult(v, 1 / vector_mag(v))


def vector_neg(v):  # :562-563
    return vec(-v[1], -v[2], -v[3])


def vector_bounce_off_plane(vector, normal):  # :568-573
    return vector_add(vector_scalar_mult(normal, 2 * vector_dot_product(normal, vector_neg(vector))), vector)


def vectors_equal(v1, v2, eps=0.0001):  # :513-521
    return (v1[1] + eps >= v2[1] and v1[1] - eps <= v2[1] and v1[2] + eps >= v2[2]
            and v1[2] - eps <= v2[2] and v1[3] + eps >= v2[3] and v1[3] - eps <= v2[3])


def _lists_max0(x):
    """lists:max([0, X]) (:275, :290): X if X > 0 else the integer 0."""
    return x if x > 0 else 0


# ---- intersections ---------------------------------------------------------------
def ray_sphere_intersect(ray, sphere):  # :364-397
    _, origin, direction = ray
    _, X0, Y0, Z0 = origin
    _, Xd, Yd, Zd = direction
    _, radius, center, _mat = sphere
    _, Xc, Yc, Zc = center
    epsilon = 0.001
    A = Xd * Xd + Yd * Yd + Zd * Zd
    B = 2 * (Xd * (X0 - Xc) + Yd * (Y0 - Yc) + Zd * (Z0 - Zc))
    C = (X0 - Xc) * (X0 - Xc) + (Y0 - Yc) * (Y0 - Yc) + (Z0 - Zc) * (Z0 - Zc) - radius * radius
    disc = B * B - 4 * A * C
    if disc >= epsilon:
        T0 = (-B + math.sqrt(disc)) / 2
        T1 = (-B - math.sqrt(disc)) / 2
        if T0 >= 0 and T1 >= 0:
            distance = T1 if T1 < T0 else T0  # lists:min([T0, T1])
            inter = vector_add(vec(X0, Y0, Z0), vector_scalar_mult(vec(Xd, Yd, Zd), distance))
            normal = vector_normalize(vector_sub(inter, vec(Xc, Yc, Zc)))
            return (distance, inter, normal)
        return None
    return None


def ray_triangle_intersect(ray, tri):  # :402-455
    _, origin, direction = ray
    _, v1, v2, v3, _mat = tri
    epsilon = 0.000001
    edge1 = vector_sub(v2, v1)
    edge2 = vector_sub(v3, v1)
    P = vector_cross_product(direction, edge2)
    det = vector_dot_product(edge1, P)
    if det < epsilon:
        return None
    T = vector_sub(origin, v1)
    U = vector_dot_product(T, P)
    if U < 0 or U > det:
        return None
    Q = vector_cross_product(T, edge1)
    V = vector_dot_product(direction, Q)
    if V < 0 or U + V > det:
        return None
    distance = vector_dot_product(edge2, Q) / det
    inter = vector_add(origin, vector_scalar_mult(direction, distance))
    normal = vector_normalize(vector_cross_product(v1, v2))
    return (distance, inter, normal)


def ray_plane_intersect(ray, plane):  # :461-480
    _, origin, direction = ray
    _, normal, dist, _mat = plane
    epsilon = 0.001
    Vd = vector_dot_product(normal, direction)
    if Vd < 0:
        V0 = -(vector_dot_product(normal, origin) + dist)
        distance = V0 / Vd
        if distance < epsilon:
            return None
        return (distance, vector_add(origin, vector_scalar_mult(direction, distance)), normal)
    return None


def ray_object_intersect(ray, obj):  # :349-359
    tag = obj[0] if isinstance(obj, tuple) and obj else None
    if tag == 'sphere':
        return ray_sphere_intersect(ray, obj)
    if tag == 'triangle':
        return ray_triangle_intersect(ray, obj)
    if tag == 'plane':
        return ray_plane_intersect(ray, obj)
    return None


def nearest_object_intersecting_ray(ray, scene):  # :300-346
    nearest, hit_loc, normal, distance = None, None, None, None  # None stands for `infinity`
    for obj in scene:
        r = ray_object_intersect(ray, obj)
        if r is not None:
            new_distance, new_hit, new_normal = r
            if distance is None or distance > new_distance:
                nearest, hit_loc, normal, distance = obj, new_hit, new_normal, new_distance
    if distance is None:
        return None
    return (nearest, distance, hit_loc, normal)


# ---- shading -------------------------------------------------------------------------
def _material(obj):  # object_*(), :575-601
    return obj[-1]


def shadow_factor(light_loc, hit_loc, obj, scene):  # :256-267
    light_vector = vector_sub(hit_loc, light_loc)
    light_direction = vector_normalize(light_vector)
    r = nearest_object_intersecting_ray(('ray', light_loc, light_direction), scene)
    if r is not None and _exact_eq(r[0], obj):
        return 1
    return 0


def diffuse_term(obj, light_loc, hit_loc, hit_normal):  # :272-279
    colour = _material(obj)[1]
    return vector_scalar_mult(('vector',) + tuple(colour[1:]),
                              _lists_max0(vector_dot_product(hit_normal,
                                                             vector_normalize(vector_sub(light_loc, hit_loc)))))


def specular_term(eye, light_loc, hit_loc, hit_normal, spec_power, shininess, spec_colour):  # :285-297
    return vector_scalar_mult(
        ('vector',) + tuple(spec_colour[1:]),
        shininess * math.pow(
            _lists_max0(vector_dot_product(
                vector_normalize(vector_add(vector_normalize(vector_sub(light_loc, hit_loc)), vector_neg(eye))),
                hit_normal)), spec_power))


def lighting_function(ray, obj, hit_loc, hit_normal, scene, depth, memo=False):  # :209-252
    final = vec(0, 0, 0)
    mat = _material(obj)
    _, _colour, spec_power, shininess, reflectivity = mat
    cached = None
    for el in scene:
        if not (isinstance(el, tuple) and el and el[0] == 'point_light'):
            continue
        _, light_colour, light_loc, spec_colour = el
        if memo and cached is not None:
            reflection = cached
        else:
            bounce = ('ray', hit_loc, vector_bounce_off_plane(ray[2], hit_normal))
            c = pixel_colour_from_ray(bounce, scene, depth - 1, memo)
            reflection = vector_scalar_mult(('vector',) + tuple(c[1:]), reflectivity)
            cached = reflection
        contribution = vector_add(diffuse_term(obj, light_loc, hit_loc, hit_normal),
                                  specular_term(ray[2], light_loc, hit_loc, hit_normal, spec_power, shininess,
                                                spec_colour))
        final = vector_add(final, vector_add(
            reflection,
            vector_scalar_mult(vector_component_mult(('vector',) + tuple(light_colour[1:]), contribution),
                               shadow_factor(light_loc, hit_loc, obj, scene))))
    return final


def pixel_colour_from_ray(ray, scene, depth, memo=False):  # :186-203
    if depth == 0:
        return ('colour', 0, 0, 0)
    r = nearest_object_intersecting_ray(ray, scene)
    if r is None:
        return ('colour', 0, 0, 0)  # ?BACKGROUND_COLOUR (:82)
    obj, _dist, hit_loc, hit_normal = r
    v = lighting_function(ray, obj, hit_loc, hit_normal, scene, depth, memo)
    return ('colour', v[1], v[2], v[3])


# ---- camera, raytracer.erl:483-511 ---------------------------------------------------
def focal_length(angle, dimension):  # :483-484
    return dimension / (2 * math.tan(angle * (math.pi / 180) / 2))


def point_on_screen(X, Y, camera):  # :486-503
    _, location, _rot, fov, screen = camera
    _, sw, sh = screen
    total = location
    for v in (vector_scalar_mult(vec(0, 0, 1), focal_length(fov, sw)),
              vec((X - 0.5) * sw, 0, 0),
              vec(0, (Y - 0.5) * sh, 0)):
        total = vector_add(v, total)
    return total


def shoot_ray(frm, through):  # :506-507
    return ('ray', frm, vector_normalize(vector_sub(through, frm)))


def ray_through_pixel(X, Y, camera):  # :510-511
    return shoot_ray(camera[1], point_on_screen(X, Y, camera))


def trace_ray_through_pixel(xy, scene, depth, memo=False):  # :180-184
    camera, rest = scene[0], scene[1:]
    c = pixel_colour_from_ray(ray_through_pixel(xy[0], xy[1], camera), rest, depth, memo)
    return (c[1], c[2], c[3])  # colour_to_pixel/1 (:613-614)


def raytraced_pixel_list_simple(width, height, scene, depth, memo=True):  # :86-99
    if width == 0 and height == 0:
        return 'done'
    if not (width > 0 and height > 0):
        raise ValueError('function_clause')
    return [(1, trace_ray_through_pixel((x / width, y / height), scene, depth, memo))
            for y in range(height) for x in range(width)]
