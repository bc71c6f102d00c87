"""CPU restatement of the reference's batch-pipeline steps around the matcher.

TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use this module as the checker; the product path
(reporter_amd.tiles, the HIP kernels) never imports it.

Each function restates one block of reference py/simple_reporter.py (Python 2):

  windows()        :144-164  per-vehicle time sort + inactivity windows (>= 2 points)
  tile_lines()     :176-196  valid-report filter, hour buckets, CSV rows per tile file
  privacy_cull()   :221-239  string sort + removal of (id, next_id) runs below `privacy`
  tile_body()      :241-253  header + rows of an uploaded tile (None when empty)

Pinning: privacy_cull/tile_body are checked against tests/golden/tiles_golden.json,
produced by running the reference's own report() (make_tiles_golden.py).  windows()
and tile_lines() live inside the reference's match() which cannot run here (it needs
the absent Valhalla matcher and Python 2's dict.iteritems), so they are a line-by-line
restatement whose parity is unpinned by reference execution.
"""
import math

INVALID_SEGMENT_ID = 0x3FFFFFFFFFFF  # simple_reporter.py:43
HEADER = ("segment_id,next_segment_id,duration,count,length,queue_length,minimum_timestamp,maximum_timestamp,"
          "source,vehicle_type")  # simple_reporter.py:252


def windows(times, inactivity=120):
    """Index ranges [i, j) of one vehicle's time-sorted points that form matching
    windows: a new window starts where the gap to the previous point exceeds
    `inactivity` (:151-153); windows of fewer than 2 points are skipped (:158-160)."""
    starts = [i for i in range(len(times)) if i == 0 or times[i] - times[i - 1] > inactivity]
    out = []
    for idx, i in enumerate(starts):
        j = starts[idx + 1] if idx + 1 < len(starts) else len(times)
        if j - i < 2:
            continue
        out.append((i, j))
    return out


def split_windows(uuids, times, inactivity=120):
    """All windows of a point stream: group by uuid, stable sort by time (:140,146),
    then windows().  Returns [(uuid, [point indices in window order])]."""
    by = {}
    for k, u in enumerate(uuids):
        by.setdefault(u, []).append(k)
    out = []
    for u in sorted(by):
        idx = sorted(by[u], key=lambda k: times[k])
        for i, j in windows([times[k] for k in idx], inactivity):
            out.append((u, idx[i:j]))
    return out


def tile_lines(reports, first_time, last_time, quantisation=3600, source="smpl_rprt", mode="auto"):
    """{tile file name: [rows]} for one matched window (:176-196).  `reports` are the
    datastore reports of report() (dicts with id, next_id?, t0, t1, length,
    queue_length); first/last_time are the window's first and last point times."""
    buckets = (last_time - first_time) // quantisation + 1            # :176 (Python 2 int division)
    tiles = {}
    keep = [r for r in reports if r["t0"] > 0 and r["t1"] > 0 and r["t1"] - r["t0"] > .5 and r["length"] > 0
            and r["queue_length"] >= 0]                                # :177
    for r in keep:
        duration = int(py2_round(r["t1"] - r["t0"]))                  # :179, Python 2 round()
        start = int(math.floor(r["t0"]))
        end = int(math.ceil(r["t1"]))
        min_bucket = start // quantisation                             # :182-183, Python 2 int division
        max_bucket = end // quantisation
        if max_bucket - min_bucket > buckets:                          # :184-187
            continue
        for b in range(min_bucket, max_bucket + 1):
            level = r["id"] & 0x7                                      # get_tile_level
            index = (r["id"] >> 3) & 0x3FFFFF                          # get_tile_index
            name = "%d_%d/%d/%d" % (b * quantisation, (b + 1) * quantisation - 1, level, index)
            row = [str(r["id"]), str(r.get("next_id", INVALID_SEGMENT_ID)), str(duration), "1", str(r["length"]),
                   str(r["queue_length"]), str(start), str(end), source, mode.upper()]
            tiles.setdefault(name, []).append(",".join(row) + "\n")
    return tiles


def py2_round(x):
    """Python 2 round(): halves away from zero (the reference runs under Python 2)."""
    return math.floor(x + 0.5) if x >= 0 else math.ceil(x - 0.5)


def privacy_cull(lines, privacy):
    """The reference's cull loop (:218-239) over the string-sorted lines, kept exact,
    including its end-of-list behaviour (the last line closes the open run with it)."""
    segments = sorted(lines)
    start = 0
    i = 0
    while i < len(segments):
        s = segments[start].split(",")
        e = segments[i].split(",")
        if s[0] != e[0] or s[1] != e[1] or i == len(segments) - 1:
            if i == len(segments) - 1:
                i += 1
            if i - start < privacy:
                segments[start:i] = []
                i = start
            else:
                start = i
        i += 1
    return segments


def tile_body(lines, privacy):
    """Uploaded text of one tile file, or None when the cull leaves nothing (:241-253)."""
    kept = privacy_cull(lines, privacy)
    if not kept:
        return None
    return HEADER + "\n" + "".join(kept)


def cull_by_groups(groups, privacy):
    """The same decision expressed over the sorted runs of equal (id, next_id):
    `groups` are the run sizes in order; returns a keep flag per run.  Every run but
    the last is kept iff its size >= privacy; the loop's end-of-list step closes the
    open run together with the final line, so a final run of ONE line is judged
    together with the run before it (and shares its fate)."""
    m = len(groups)
    keep = [g >= privacy for g in groups]
    if m == 1:
        return keep
    if groups[-1] == 1:
        k = groups[-2] + 1 >= privacy
        keep[-2] = k
        keep[-1] = k
    return keep
