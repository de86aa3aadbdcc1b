"""Row-band split host logic (acmmp/band.py): bands cover the view, each spans >= the 23-row halo."""
import pytest

from acmmp import band


@pytest.mark.parametrize("H,n", [(1500, 1), (1500, 2), (1500, 8), (97, 4), (65, 2), (100, 9), (22, 3), (2133, 8)])
def test_split_rows_cover_and_span_halo(H, n):
    bands = band.split_rows(H, n)
    assert bands[0][0] == 0 and bands[-1][1] == H
    assert all(a[1] == b[0] for a, b in zip(bands, bands[1:]))
    assert len(bands) <= n
    if len(bands) > 1:
        assert all(hi - lo >= band.HALO for lo, hi in bands)
    sizes = [hi - lo for lo, hi in bands]
    assert max(sizes) - min(sizes) <= 1


def test_split_rows_caps_band_count():
    assert len(band.split_rows(100, 9)) == 4          # 100 // 23
    assert band.split_rows(22, 3) == [(0, 22)]
    with pytest.raises(ValueError):
        band.split_rows(0, 2)
