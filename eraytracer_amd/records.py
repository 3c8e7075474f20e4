"""The reference's records as Erlang-style tuples (raytracer.erl:72-84) and its
default scene (raytracer.erl:616-665).

``vector(4, 0, 10)`` is ``(Atom('vector'), 4, 0, 10)`` — the term ``{vector,4,0,10}``
that ``#vector{x=4, y=0, z=10}`` denotes.  Numbers keep the int/float type the
reference source gives them (``scene_test/0``, raytracer.erl:760-801, pins it).
"""
from __future__ import annotations

from .terms import Atom

__all__ = [
    "vector", "colour", "ray", "screen", "camera", "material", "sphere", "triangle", "plane",
    "point_light", "scene", "BACKGROUND_COLOUR", "UNKNOWN_COLOUR", "FOG_DISTANCE", "tag",
]

VECTOR, COLOUR, RAY, SCREEN, CAMERA = Atom("vector"), Atom("colour"), Atom("ray"), Atom("screen"), Atom("camera")
MATERIAL, SPHERE, TRIANGLE, PLANE = Atom("material"), Atom("sphere"), Atom("triangle"), Atom("plane")
POINT_LIGHT = Atom("point_light")


def vector(x, y, z):  # -record(vector, {x, y, z}).              :72
    return (VECTOR, x, y, z)


def colour(r, g, b):  # -record(colour, {r, g, b}).              :73
    return (COLOUR, r, g, b)


def ray(origin, direction):  # -record(ray, {origin, direction}).  :74
    return (RAY, origin, direction)


def screen(width, height):  # -record(screen, {width, height}).    :75
    return (SCREEN, width, height)


def camera(location, rotation, fov, screen_):  # -record(camera, {location, rotation, fov, screen}).  :76
    return (CAMERA, location, rotation, fov, screen_)


def material(colour_, specular_power, shininess, reflectivity):  # :77
    return (MATERIAL, colour_, specular_power, shininess, reflectivity)


def sphere(radius, center, material_):  # -record(sphere, {radius, center, material}).  :78
    return (SPHERE, radius, center, material_)


def triangle(v1, v2, v3, material_):  # -record(triangle, {v1, v2, v3, material}).  :79
    return (TRIANGLE, v1, v2, v3, material_)


def plane(normal, distance, material_):  # -record(plane, {normal, distance, material}).  :80
    return (PLANE, normal, distance, material_)


def point_light(diffuse_colour, location, specular_colour):  # :81
    return (POINT_LIGHT, diffuse_colour, location, specular_colour)


BACKGROUND_COLOUR = colour(0, 0, 0)  # :82
UNKNOWN_COLOUR = colour(0, 1, 0)     # :83 (unused by the reference)
FOG_DISTANCE = 40                    # :84 (unused by the reference)


def tag(term):
    """The record tag of a term, or None."""
    if isinstance(term, tuple) and term and isinstance(term[0], Atom):
        return term[0]
    return None


def scene():
    """scene/0 (raytracer.erl:618-665): camera first, then lights and objects."""
    return [
        camera(vector(0, 0, -2), vector(0, 0, 0), 90, screen(4, 3)),
        point_light(colour(1, 1, 0.5), vector(5, -2, 0), colour(1, 1, 1)),
        point_light(colour(1, 0, 0.5), vector(-10, 0, 7), colour(1, 0, 0.5)),
        sphere(4, vector(4, 0, 10), material(colour(0, 0.5, 1), 20, 1, 0.1)),
        sphere(4, vector(-5, 3, 9), material(colour(1, 0.5, 0), 4, 0.25, 0.5)),
        sphere(4, vector(-4.5, -2.5, 14), material(colour(0.5, 1, 0), 20, 0.25, 0.7)),
        triangle(vector(-2, 5, 5), vector(4, 5, 10), vector(4, -5, 10),
                 material(colour(1, 0.5, 0), 4, 0.25, 0.5)),
        plane(vector(0, -1, 0), 5, material(colour(1, 1, 1), 1, 0, 0.01)),
    ]
