"""Scene entry points of src/scenes.rs, built by the C++ host (seeded; the reference uses thread_rng)."""
from __future__ import annotations

from .scene import SceneBuilder

SCENES = ("random", "random-night", "demo", "perlin", "earth", "box-light", "cornell", "spheres", "final")


def random_scene(seed: int = 0x5EED, night: bool = False) -> SceneBuilder:  # scenes.rs:281-429
    return SceneBuilder.builtin("random-night" if night else "random", seed)


def create_cornell_box() -> SceneBuilder:  # scenes.rs:23-63
    return SceneBuilder.builtin("cornell")


def create_perlin_demo() -> SceneBuilder:  # scenes.rs:65-79
    return SceneBuilder.builtin("perlin")


def create_earth_demo() -> SceneBuilder:  # scenes.rs:81-93
    return SceneBuilder.builtin("earth")


def create_box_light() -> SceneBuilder:  # scenes.rs:94-127
    return SceneBuilder.builtin("box-light")


def create_scene() -> SceneBuilder:  # scenes.rs:431-483 (render demo)
    return SceneBuilder.builtin("demo")


def gen_spheres(seed: int = 0xDEADBEEF, side_len: int = 11) -> SceneBuilder:
    """benches/my_benchmark.rs:35-60 gen_spheres (22^3 = 10,648 spheres at side 11) with random book-1
    materials: the stand-in for BASELINE config 5 (no ~10k-primitive scene exists in the reference)."""
    return SceneBuilder.builtin(f"spheres:{side_len}", seed)


def final_scene(seed: int = 0x5EED, n_ground: int = 20, n_cluster: int = 1000) -> SceneBuilder:
    """Book 2 ("The Next Week") final_scene, BASELINE config 5: needs the book-2 extensions
    (moving sphere, constant media, instance transform) that the reference does not have."""
    return SceneBuilder.builtin(f"final:{n_ground}:{n_cluster}", seed)
