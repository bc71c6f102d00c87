"""Stage-by-stage comparison of the HIP engine against the CPU oracle."""
import numpy as np


def state_slots(trace_off, n_states):
    """Boolean mask of point slots that hold a state layer."""
    P = int(trace_off[-1])
    m = np.zeros(P, bool)
    for k in range(len(trace_off) - 1):
        o = int(trace_off[k])
        m[o:o + int(n_states[k])] = True
    return m


def compare_all(gpu, ref, trace_off, check_reports=True):
    """Assert bit-exact agreement of every stage; returns a dict of counts."""
    n_states, orig = gpu.states()
    np.testing.assert_array_equal(n_states, ref["n_states"], "n_states")
    sm = state_slots(trace_off, n_states)
    np.testing.assert_array_equal(orig[sm], ref["state_orig"][sm], "state_orig")

    cn, road, s, sq = gpu.candidates()
    np.testing.assert_array_equal(cn[sm], ref["cand_n"][sm], "cand_n")
    kmask = np.arange(16)[None, :] < cn[:, None]
    kmask &= sm[:, None]
    np.testing.assert_array_equal(road[kmask], ref["cand_road"][kmask], "cand_road")
    np.testing.assert_array_equal(s[kmask], ref["cand_s"][kmask], "cand_s")
    np.testing.assert_array_equal(sq[kmask].view(np.uint32), ref["cand_sq"][kmask].view(np.uint32), "cand_sq bits")

    toff, gc, route = gpu.routes()
    first = np.zeros(len(sm), bool)
    first[trace_off[:-1][n_states > 0]] = True
    tm = sm & ~first
    np.testing.assert_array_equal(toff[tm], ref["trans_off"][tm], "trans_off")
    np.testing.assert_array_equal(gc[tm].view(np.uint64), ref["gc"][tm].view(np.uint64), "gc bits")
    np.testing.assert_array_equal(route, ref["route"], "route_cm")

    choice, cs = gpu.viterbi()
    np.testing.assert_array_equal(cs[sm], ref["chain_start"][sm], "chain_start")
    np.testing.assert_array_equal(choice[sm], ref["choice"][sm], "choice")

    poff, pcnt, pool, rdist = gpu.paths()
    inchain = tm & (cs == 0) & (choice >= 0)
    np.testing.assert_array_equal(pcnt[inchain], ref["path_cnt"][inchain], "path_cnt")
    np.testing.assert_array_equal(rdist[inchain], ref["route_dist"][inchain], "route_dist")
    for p in np.nonzero(inchain)[0]:
        a = pool[poff[p]:poff[p] + pcnt[p]]
        b = ref["path_pool"][ref["path_off"][p]:ref["path_off"][p] + ref["path_cnt"][p]]
        if not np.array_equal(a, b):
            raise AssertionError("path edges differ at slot %d: gpu %s oracle %s" % (p, a, b))

    soff, segs = gpu.segments()
    np.testing.assert_array_equal(soff, ref["seg_off"], "seg_off")
    if len(segs):
        for f in segs.dtype.names:
            a, b = segs[f], ref["segs"][f]
            if a.dtype.kind == "f":
                a, b = a.view(np.uint64), b.view(np.uint64)
            np.testing.assert_array_equal(a, b, "segments." + f)
    return dict(points=int(trace_off[-1]), states=int(sm.sum()), transitions=len(route),
                chained=int(inchain.sum()), segments=len(segs))
