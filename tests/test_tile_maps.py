"""The XCD-grouped tile order of csrc/precond_gemm.hip (template flag XCD),
transcribed line for line: for every problem shape it must be a bijection
onto the tile grid (a hole or a repeat would leave output tiles unwritten or
written twice), and tiles sharing the larger operand's panel must get block
indices equal mod 8 (one XCD) wherever a full group of 8 panels exists."""
import pytest


def xcd_tile(local, tiles_m, tiles_n):
    by_a = tiles_m >= tiles_n
    np_, other = (tiles_m, tiles_n) if by_a else (tiles_n, tiles_m)
    full = (np_ // 8) * 8 * other
    if local < full:
        i = local >> 3
        pa = 8 * (i // other) + (local & 7)
        ob = i % other
    else:
        r = local - full
        pa = (np_ // 8) * 8 + r // other
        ob = r % other
    return (pa, ob) if by_a else (ob, pa)


@pytest.mark.parametrize('tiles_m', list(range(1, 41)))
def test_xcd_tile_order_is_a_bijection(tiles_m):
    for tiles_n in range(1, 41):
        n = tiles_m * tiles_n
        seen = set(xcd_tile(l, tiles_m, tiles_n) for l in range(n))
        assert len(seen) == n
        assert all(0 <= tm < tiles_m and 0 <= tn < tiles_n for tm, tn in seen)


@pytest.mark.parametrize('tiles_m,tiles_n,begin', [(36, 4, 0), (36, 4, 13), (4, 36, 5),
                                                    (16, 16, 3), (9, 2, 7)])
def test_xcd_tile_order_keeps_panels_on_one_xcd(tiles_m, tiles_n, begin):
    by_a = tiles_m >= tiles_n
    np_ = tiles_m if by_a else tiles_n
    xcd_of_panel = {}
    for local in range(tiles_m * tiles_n):
        tm, tn = xcd_tile(local, tiles_m, tiles_n)
        panel = tm if by_a else tn
        if panel >= (np_ // 8) * 8:
            continue                      # the row-major remainder
        x = (begin + local) % 8           # blocks are dealt round-robin over 8 XCDs
        assert xcd_of_panel.setdefault(panel, x) == x
    if np_ >= 8:
        assert len(set(xcd_of_panel.values())) == 8   # every XCD gets panels
