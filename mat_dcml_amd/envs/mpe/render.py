"""RGB frames of the batched MPE worlds and GIF export (the reference renders through its pyglet viewer and
``imageio.mimsave``, ``mat_src/mat/runner/shared/mpe_runner.py:193-254``; neither pyglet nor imageio exists here, so
frames are rasterised with numpy and written with Pillow).

Camera as the reference's shared viewer: centred on the origin, ``cam_range`` = 1 world unit to each edge.  Entities
are filled discs of their collision size; colours follow the reference scenarios' scheme (good agents blue,
adversaries red, landmarks grey).
"""
from __future__ import annotations

import numpy as np

AGENT_RGB = (0.35, 0.35, 0.85)
ADVERSARY_RGB = (0.85, 0.35, 0.35)
LANDMARK_RGB = (0.25, 0.25, 0.25)


def render_frame(world, env_index: int = 0, size: int = 400, cam_range: float = 1.0) -> np.ndarray:
    """(size, size, 3) uint8 frame of env ``env_index`` of a ``core.World``."""
    t = world.t
    pos = world.pos[env_index].detach().float().cpu().numpy()            # (N, 2)
    rad = t.size.detach().float().cpu().numpy()
    adv = t.adversary.detach().cpu().numpy()
    img = np.ones((size, size, 3), dtype=np.float32)
    ys, xs = np.mgrid[0:size, 0:size].astype(np.float32)
    scale = 0.5 * size / cam_range
    # landmarks below agents (the reference draws world.entities in order; agents overlap landmarks when they
    # sit on them, which is the informative case)
    order = list(range(t.nA, t.nA + t.nL)) + list(range(t.nA))
    for i in order:
        cx = size * 0.5 + pos[i, 0] * scale
        cy = size * 0.5 - pos[i, 1] * scale                               # world +y is up
        r = max(rad[i] * scale, 1.0)
        inside = (xs - cx) ** 2 + (ys - cy) ** 2 <= r * r
        if i < t.nA:
            rgb = ADVERSARY_RGB if adv[i] else AGENT_RGB
        else:
            rgb = LANDMARK_RGB
        img[inside] = rgb
    return (img * 255.0 + 0.5).astype(np.uint8)


def save_gif(frames, path: str, ifi: float) -> None:
    """Animated GIF, ``ifi`` seconds per frame (``imageio.mimsave(..., duration=ifi)`` in the reference)."""
    from PIL import Image
    ims = [Image.fromarray(f) for f in frames]
    ims[0].save(path, save_all=True, append_images=ims[1:], duration=max(int(round(ifi * 1000)), 1), loop=0)
