"""Top-down RGB frames of one env from device state (`mas_render_view`), for
debugging and GIFs of GPU rollouts -- the `rgb_array` mode of the
reference's renderer (`rendering.py:118-613`, pygame), restated as a small
numpy rasterizer.  It draws what the reference draws at the body level:
walls, the safe zone, boxes, box items, heals and agents with a heading
tick and a health bar; teams are coloured when the config has two teams.
Colours and line styles are this build's, not pygame's.  No display
('human' mode needs pygame, which this build does not have)."""
from typing import Any, Dict, Optional

import numpy as np

WALL = (60, 60, 60)
ZONE = (40, 170, 40)
BOX = (150, 100, 50)
ITEM = (210, 170, 110)
HEAL = (220, 40, 40)
AGENTS = [(40, 90, 220), (230, 140, 20), (140, 60, 200), (30, 170, 170),
          (200, 60, 140), (120, 120, 30), (90, 90, 90), (20, 120, 60)]
TEAMS = [(40, 90, 220), (230, 140, 20)]
BACKGROUND = (245, 245, 240)


class _Canvas:
    def __init__(self, size: int, half: float):
        self.img = np.empty((size, size, 3), dtype=np.uint8)
        self.img[:] = BACKGROUND
        self.size, self.scale = size, size / (2.0 * half)
        self.half = half
        ys, xs = np.mgrid[0:size, 0:size]
        # world coordinates of the pixel centres (y up)
        self.wx = (xs + 0.5) / self.scale - half
        self.wy = half - (ys + 0.5) / self.scale

    def fill(self, mask, colour):
        self.img[mask] = colour

    def rect(self, cx, cy, hx, hy, angle, colour):
        c, s = np.cos(angle), np.sin(angle)
        dx, dy = self.wx - cx, self.wy - cy
        lx, ly = c * dx + s * dy, -s * dx + c * dy
        self.fill((np.abs(lx) <= hx) & (np.abs(ly) <= hy), colour)

    def disc(self, cx, cy, r, colour):
        self.fill((self.wx - cx) ** 2 + (self.wy - cy) ** 2 <= r * r, colour)

    def ring(self, cx, cy, r, width, colour):
        d = np.sqrt((self.wx - cx) ** 2 + (self.wy - cy) ** 2)
        self.fill(np.abs(d - r) <= width, colour)

    def segment(self, x0, y0, x1, y1, width, colour):
        ex, ey = x1 - x0, y1 - y0
        L2 = ex * ex + ey * ey
        t = np.clip(((self.wx - x0) * ex + (self.wy - y0) * ey) / max(L2, 1e-12), 0.0, 1.0)
        px, py = x0 + t * ex - self.wx, y0 + t * ey - self.wy
        self.fill(px * px + py * py <= width * width, colour)


def render_rgb(view: Dict[str, Any], size: int = 400, teams: bool = False, agent_r: float = 0.5,
               heal_r: float = 0.25) -> np.ndarray:
    """uint8 [size, size, 3] top-down frame of a parsed mas_render_view."""
    half = 0.5 * view['floor_size'] + 1.0
    cv = _Canvas(size, half)
    zx, zy, zr = (float(x) for x in view['zone'])
    if zr > 0:
        cv.ring(zx, zy, zr, 1.0 / cv.scale, ZONE)
    for x, y, a, hx, hy in view['walls']:
        cv.rect(x, y, hx, hy, a, WALL)
    for x, y, hx, hy, _ in view['boxes']:
        cv.rect(x, y, hx, hy, 0.0, BOX)
    for x, y, hx, hy in view['items']:
        cv.rect(x, y, 0.5 * hx, 0.5 * hy, 0.0, ITEM)
    for x, y in view['heals']:
        cv.disc(x, y, heal_r, HEAL)
    A = len(view['agents'])
    for i, (x, y, a, alive, health) in enumerate(view['agents']):
        if alive < 0.5:
            continue
        col = TEAMS[int(i >= A // 2)] if teams else AGENTS[i % len(AGENTS)]
        cv.disc(x, y, agent_r, col)
        cv.segment(x, y, x + agent_r * np.cos(a), y + agent_r * np.sin(a), 1.5 / cv.scale, (255, 255, 255))
        frac = float(np.clip(health / 100.0, 0.0, 1.0))
        bar_y = y + agent_r + 0.25
        cv.rect(x, bar_y, agent_r, 0.08, 0.0, (200, 200, 200))
        if frac > 0:
            cv.rect(x - agent_r * (1 - frac), bar_y, agent_r * frac, 0.08, 0.0, (40, 180, 40))
    return cv.img


def render_env(vec_env, env: int = 0, size: int = 400, teams: Optional[bool] = None) -> np.ndarray:
    """Frame of env `env` of a VecMaSurvival (synchronises with the device)."""
    view = vec_env.render_view(env)
    if teams is None:
        teams = bool(getattr(vec_env.rc, 'has_teams', False))
    return render_rgb(view, size=size, teams=teams)
