"""Host model of the path kernel's lane -> pixel mapping (bdpt_kernels.hip, BDPT_PACK_EDGES): the
regular 32x8 workgroup tiles plus the packed frame edges (the last workgroup column when it holds
<= 8 columns, the last workgroup row when it holds < 8 rows) cover every pixel exactly once.  The
GPU parity tests check the kernel itself against the oracle on these frame shapes."""
import pytest

BTW, BTH, WTW, WX = 32, 8, 8, 4


def cover(W, H):
    gx, gy = (W + BTW - 1) // BTW, (H + BTH - 1) // BTH
    xt, yt = (gx - 1) * BTW, (gy - 1) * BTH
    tw, th = W - xt, H - yt
    seen = {}
    for bx in range(gx):
        for by in range(gy):
            for t in range(256):
                lane, wave = t & 63, t >> 6
                x = bx * BTW + (wave % WX) * WTW + (lane % WTW)
                ly = by * BTH + (wave // WX) * 8 + (lane // WTW)
                if tw <= WTW and bx == gx - 1:
                    q = by * 256 + t
                    x, ly = xt + q % tw, q // tw
                elif th < BTH and bx < gx - 1 and by == gy - 1:
                    q = bx * 256 + t
                    x, ly = q % xt, yt + q // xt
                if x < W and ly < H:
                    seen[(x, ly)] = seen.get((x, ly), 0) + 1
    return seen


@pytest.mark.parametrize("W,H", [(1921, 1081), (121, 89), (1, 1), (1, 301), (1921, 1), (37, 9), (65, 49),
                                 (33, 17), (97, 65), (32, 8), (40, 8), (33, 8), (8, 3), (9, 3), (64, 64),
                                 (513, 513), (257, 193)])
def test_every_pixel_once(W, H):
    seen = cover(W, H)
    assert len(seen) == W * H and all(v == 1 for v in seen.values())
