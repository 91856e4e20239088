"""Render-harness host pieces (run.py:80-356 counterparts, apn_amd.harness): the PNG writer /
reader round trip, the skeleton overlay rasteriser, the mip-NeRF SSIM. CPU only."""
import numpy as np

from apn_amd import harness as Hn


def test_png_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    for shape in [(7, 5, 3), (4, 9), (3, 3, 4)]:
        img = rng.integers(0, 256, shape, dtype=np.uint8)
        p = tmp_path / f"x{len(shape)}.png"
        Hn.write_png(p, img)
        back = Hn.read_png(p)
        assert np.array_equal(back.reshape(img.shape), img)
        assert open(p, "rb").read(8) == b"\x89PNG\r\n\x1a\n"


def test_to8b_clips_and_truncates():
    x = np.array([-0.5, 0.0, 0.5, 0.999, 1.0, 2.0])
    assert Hn.to8b(x).tolist() == [0, 0, 127, 254, 255, 255]


def test_draw_skeleton_lines_and_discs():
    img = np.ones((20, 30, 3))
    joints = np.array([[2, 3], [12, 3], [12, 15]], np.int32)   # (x, y)
    Hn.draw_skeleton(img, joints, [[0, 1], [1, 2]])
    assert (img[3, 2:13] == 0).all()                 # horizontal bone on row y = 3
    assert (img[3:16, 12] == 0).all()                # vertical bone on column x = 12
    assert (img[15, 9:16] == 0).all() and img[15, 16, 0] == 1.0   # disc of radius 3 around (12, 15)
    assert img[10, 5, 0] == 1.0                      # away from the skeleton untouched
    far = np.ones((4, 4, 3))
    Hn.draw_skeleton(far, np.array([[-5, 2], [100, 2]], np.int32), [[0, 1]])   # clipped to the image
    assert (far[2] == 0).all() and (far[0] == 1).all()


def test_draw_line_closed_form_equals_walk():
    """The vectorised line rasteriser draws exactly the pixels of the error-term walk, every octant,
    degenerate and clipped lines included."""
    rng = np.random.default_rng(7)
    for _ in range(3000):
        x0, y0, x1, y1 = (int(v) for v in rng.integers(-15, 45, 4))
        a, b = np.ones((30, 30)), np.ones((30, 30))
        Hn._draw_line(a, (x0, y0), (x1, y1), 0.0)
        Hn._draw_line_walk(b, (x0, y0), (x1, y1), 0.0)
        assert np.array_equal(a, b), (x0, y0, x1, y1)


def test_rgb_ssim():
    rng = np.random.default_rng(1)
    a = rng.uniform(0, 1, (32, 40, 3))
    assert abs(Hn.rgb_ssim(a, a, 1.0) - 1.0) < 1e-12
    b = np.clip(a + rng.normal(0, 0.05, a.shape), 0, 1)
    c = np.clip(a + rng.normal(0, 0.2, a.shape), 0, 1)
    s_b, s_c = Hn.rgb_ssim(a, b, 1.0), Hn.rgb_ssim(a, c, 1.0)
    assert 1.0 > s_b > s_c > 0.0
    m = Hn.rgb_ssim(a, b, 1.0, return_map=True)
    assert m.shape == (32 - 10, 40 - 10, 3)
