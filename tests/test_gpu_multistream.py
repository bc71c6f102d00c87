"""engine.MultiMatcher / rm_runners_rerun: one batch as concurrent parts on their own HIP
streams (what bench.py runs by default) gives exactly the single-stream results: the same
segments per trace, reports and speed histogram, on every rerun."""
import numpy as np
import pytest

from reporter_amd import dist, engine, world

pytestmark = pytest.mark.gpu


def _segments_of(m):
    if isinstance(m, engine.BatchMatcher):
        return [m.segments()]
    return [bm.segments() for bm in m.bms]


def _flat(parts):
    offs, segs, base = [np.zeros(1, np.uint64)], [], 0
    for off, s in parts:
        offs.append(off[1:].astype(np.uint64) + base)
        base += int(off[-1])
        segs.append(s)
    return np.concatenate(offs), np.concatenate(segs)


@pytest.mark.parametrize("parts", [2, 3])
def test_multistream_equals_single(small_world, parts):
    tr = world.generate_traces(small_world, n_traces=120, n_points=300, rate_s=1.0, noise_m=5.0, seed=21)
    eng = engine.Engine(small_world, 0)
    opts = engine.default_options(1)
    nbytes = eng.n_segments * 16 * 4
    h1, h2 = dist.DeviceBuffer(nbytes), dist.DeviceBuffer(nbytes)
    single = engine.BatchMatcher(eng)
    single.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, hist_dev=h1.ptr, zero_hist=True)
    multi = engine.MultiMatcher(eng, parts)
    multi.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, hist_dev=h2.ptr, zero_hist=True)
    assert len(multi.bms) == parts
    o1, s1 = _flat(_segments_of(single))
    for rep in range(3):
        if rep:
            multi.rerun(hist_dev=h2.ptr, zero_hist=True)
        o2, s2 = _flat(_segments_of(multi))
        assert np.array_equal(o1, o2)
        assert s1.tobytes() == s2.tobytes()
        assert np.array_equal(h1.download(), h2.download())
        a, b = single.sizes(), multi.sizes()
        for k in ("points", "traces", "transitions", "path_edges", "segments", "reports"):
            assert a[k] == b[k], k
    multi.close(); single.close(); h1.close(); h2.close(); eng.close()
