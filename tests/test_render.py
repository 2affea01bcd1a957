"""Frames from device state: the rasterizer on a
synthetic render view (CPU), and mas_render_view + MaSurvival.render on the
GPU."""
import numpy as np
import pytest

from masurvival.render import AGENTS, BACKGROUND, BOX, WALL, render_rgb
from masurvival.vec_env import MAS_RENDER_VIEW_FLOATS, parse_render_view


def _view(agents, boxes=(), floor=20.0):
    v = np.zeros(MAS_RENDER_VIEW_FLOATS, dtype=np.float32)
    AM, BM, HM = 4, 4, 4
    v[0], v[1], v[7], v[8], v[9], v[10] = len(agents), len(boxes), AM, BM, HM, floor
    v[4:7] = (0.0, 0.0, 0.0)
    walls = [(-10.1, 0.0, 0.0, 0.1, 10.0), (0.0, 10.1, np.pi / 2, 0.1, 10.0),
             (10.1, 0.0, 0.0, 0.1, 10.0), (0.0, -10.1, np.pi / 2, 0.1, 10.0)]
    v[12:32] = np.array(walls, dtype=np.float32).reshape(-1)
    for i, a in enumerate(agents):
        v[32 + 5 * i:32 + 5 * i + 5] = a
    for b, box in enumerate(boxes):
        o = 32 + 5 * AM + 5 * b
        v[o:o + 5] = box
    return parse_render_view(v)


def _px(img_size, floor, x, y):
    half = 0.5 * floor + 1.0
    s = img_size / (2 * half)
    return int((half - y) * s), int((x + half) * s)  # row, col


def test_rasterizer_draws_bodies_where_they_are():
    view = _view([(-5.0, 3.0, 0.0, 1.0, 100.0), (4.0, -4.0, 1.0, 0.0, 0.0)], boxes=[(2.0, 2.0, 0.5, 0.5, 20.0)])
    assert len(view['agents']) == 2 and len(view['boxes']) == 1
    img = render_rgb(view, size=200)
    assert img.shape == (200, 200, 3) and img.dtype == np.uint8
    r, c = _px(200, 20.0, -5.0 - 0.3, 3.0 - 0.3)  # inside agent 0, off its heading tick
    assert tuple(img[r, c]) == AGENTS[0]
    r, c = _px(200, 20.0, 4.0 - 0.3, -4.0 - 0.3)  # agent 1 is dead: not drawn
    assert tuple(img[r, c]) == BACKGROUND
    r, c = _px(200, 20.0, 2.0, 2.0)
    assert tuple(img[r, c]) == BOX
    r, c = _px(200, 20.0, -10.1, 0.0)
    assert tuple(img[r, c]) == WALL


@pytest.mark.gpu
def test_render_view_and_frame_on_gpu():
    from masurvival.config import C3_CONFIG
    from masurvival.envs.masurvival_env import MaSurvival
    from masurvival.vec_env import VecMaSurvival
    env = VecMaSurvival(C3_CONFIG, n_envs=8, seeds=range(8))
    env.reset()
    for e in range(8):
        v = env.render_view(e)
        assert len(v['agents']) == 4
        assert np.all(v['agents'][:, 3] == 1.0) and np.all(v['agents'][:, 4] == 100.0)
        assert np.all(np.abs(v['agents'][:, :2]) < 0.5 * v['floor_size'])
        assert v['floor_size'] > 0 and v['walls'].shape == (4, 5)
    env.close()
    single = MaSurvival()
    single.reset(seed=0)
    frame = single.render(mode='rgb_array')
    assert frame.shape == (400, 400, 3) and frame.dtype == np.uint8
    assert (frame != np.array(BACKGROUND, dtype=np.uint8)).any()
    with pytest.raises(NotImplementedError):
        single.render(mode='human')
    single.close()
