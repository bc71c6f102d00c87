"""ORACLE — test infrastructure only.  Never imported by the product path.

CPU restatement of the reference's post-match step ``report()``
(/root/reference/py/reporter_service.py:79-179).  Used only by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg, as the
checker for the GPU report epilogue (kernel A8 in DESIGN.md).

Parity: PINNED.  ``tests/test_report_oracle.py`` checks this restatement
against ``tests/golden/report_golden.json``, produced by running the
reference's own ``report()`` (tests/golden/make_report_golden.py).

The behaviours reproduced, with the line they follow:
  * tail trim: walk back while ``end - start_time < threshold`` (86-87)
  * ``shape_used`` = begin_shape_index at the trimmed index, omitted when 0 (89-92, 165)
  * only *prior* segments are emitted; the last kept index never is (103-158)
  * emit iff prior has an id, prior_length > 0 and current is not internal (122)
  * t1 / next_id from the current segment when its level is a transition level (125-127)
  * invalid time: dt <= 0, inf or nan (131-132); invalid speed: 3.6*len/dt > 160 (133-134)
  * successful/unreported lengths are ASSIGNED (last wins), km rounded to 3 dp (138, 142)
  * internal segments after the first keep the previous prior (145-147)
  * discontinuity: start == -1 and previous end == -1 (115-116)
  * unassociated: no id and not internal (161-162)
"""
import math

SPEED_LIMIT_KPH = 160.0  # reporter_service.py:133


def _level(seg_id):
    # reporter_service.py:119 — level lives in the low 3 bits; no id -> -1
    return -1 if seg_id is None else (seg_id & 0x7)


def trim_index(segments, trace_end_time, threshold_sec):
    """Index of the last segment that may carry a report (reporter_service.py:86-87)."""
    k = len(segments) - 1
    while k >= 0 and trace_end_time - segments[k]["start_time"] < threshold_sec:
        k -= 1
    return k


def report(match, trace, threshold_sec, report_levels, transition_levels):
    segs = match["segments"]
    end_time = trace["trace"][-1]["time"]
    last = trim_index(segs, end_time, threshold_sec)
    shape_used = segs[last]["begin_shape_index"] if last >= 0 else None

    match["mode"] = "auto"  # reporter_service.py:96 (hard-coded)
    stats = dict(ok=0, unrep=0, ok_len=0, unrep_len=0, disc=0, bad_time=0, bad_speed=0, unassoc=0)
    reports = []
    prior = None  # dict(id, t0, t_end, length, level, queue)

    for k in range(last + 1):
        seg = segs[k]
        sid = seg.get("segment_id")
        st = seg.get("start_time")
        en = seg.get("end_time")
        internal = seg.get("internal", False)
        if k > 0 and seg["start_time"] == -1 and segs[k - 1]["end_time"] == -1:
            stats["disc"] += 1
        lvl = _level(sid)

        if prior is not None and prior["id"] is not None and prior["length"] > 0 and internal != True:
            if prior["level"] in report_levels:
                to_next = lvl in transition_levels
                rec = {"id": prior["id"], "t0": prior["t0"], "t1": st if to_next else prior["t_end"],
                       "length": prior["length"], "queue_length": prior["queue"]}
                if to_next and sid is not None:
                    rec["next_id"] = sid
                dt = float(rec["t1"]) - float(rec["t0"])
                if dt <= 0 or math.isinf(dt) or math.isnan(dt):
                    stats["bad_time"] += 1
                elif (prior["length"] / dt) * 3.6 > SPEED_LIMIT_KPH:
                    stats["bad_speed"] += 1
                else:
                    reports.append(rec)
                    stats["ok"] += 1
                    stats["ok_len"] = round(prior["length"] * 0.001, 3)
            else:
                stats["unrep"] += 1
                stats["unrep_len"] = round(prior["length"] * 0.001, 3)

        if not (internal == True and k != 0):
            prior = {"id": sid, "t0": st, "t_end": en, "length": seg.get("length"),
                     "level": lvl, "queue": seg.get("queue_length")}
        if sid is None and internal == False:
            stats["unassoc"] += 1

    out = {"stats": {
        "successful_matches": {"count": stats["ok"], "length": stats["ok_len"]},
        "unreported_matches": {"count": stats["unrep"], "length": stats["unrep_len"]},
        "match_errors": {"discontinuities": stats["disc"], "invalid_speeds": stats["bad_speed"],
                         "invalid_times": stats["bad_time"]},
        "unassociated_segments": stats["unassoc"]}}
    if shape_used:
        out["shape_used"] = shape_used
    out["segment_matcher"] = match
    out["datastore"] = {"mode": "auto", "reports": reports}
    return out


def valid_for_tile(r):
    """Batch-pipeline filter on a report (simple_reporter.py:177)."""
    return (r["t0"] > 0 and r["t1"] > 0 and r["t1"] - r["t0"] > 0.5
            and r["length"] > 0 and r["queue_length"] >= 0)
