"""Grader.sh's scoring, restated in Python (the reference's only automated test).

Follows /root/reference/Grader.sh: the same `grep` (regex, substring) / `cut -d" "` /
`sort -u` / `awk '{print $1}'` semantics per scenario, the same point values:
  single failure  (Grader.sh:29-76)   join 10, completeness 10, accuracy 10
  multi failure   (Grader.sh:77-139)  join 10, completeness 2 per failed node (>= 5 removals),
                                      accuracy 2 per failed node (exactly 20 other removals)
  drop + single   (Grader.sh:140-190) join 15, completeness 15 (accuracy commented out)
Maximum 90.  The shell script itself cannot travel to the GPU box (the reference tree is
not there), so tests use this restatement; tests/test_oracle_golden.py checks it scores
every golden run of the reference 30/30/30.
"""
import re


def _lines(dbg):
    return dbg.decode().split("\n")


def _grep(lines, pat):
    rx = re.compile(pat)
    return [l for l in lines if rx.search(l)]


def _join_points(lines, pts):
    joined = _grep(lines, "joined")
    pairs = set()
    for l in joined:
        f = l.split(" ")
        pairs.add((f[1], " ".join(f[3:7])))
    if len(pairs) == 100:
        return pts
    cnt = 0
    for i in sorted(set(l.split(" ")[1] for l in joined)):
        mine = _grep(joined, "^ " + i)
        rest = [" ".join(l.split(" ")[3:7]) for l in mine]
        rest = set(r for r in rest if not re.search(i, r))
        if len(rest) == 9:
            cnt += 1
    return pts if cnt == 10 else 0


def _failed_nodes(lines):
    uniq = sorted(set(_grep(lines, "Node failed at time")))
    return [l.split()[0] for l in uniq]


def score(dbg, scenario):
    lines = _lines(dbg)
    removed = sorted(set(_grep(lines, "removed")))
    failed = _failed_nodes(lines)
    if scenario == "singlefailure":
        pts = _join_points(lines, 10)
        fn = failed[0]
        failcount = len(_grep(removed, fn))
        pts += 10 if failcount >= 9 else 0
        acc = len([l for l in removed if not re.search(fn, l)])
        pts += 10 if acc == 0 and failcount > 0 else 0
        return pts
    if scenario == "multifailure":
        pts = _join_points(lines, 10)
        tmp = cnt = 0
        for i in failed:
            if len(_grep(removed, i)) >= 5:
                tmp += 2
            cnt += 1
            if cnt > 5:
                break
        pts += tmp
        tmp = 0
        for i in failed:
            if len([l for l in removed if not re.search(i, l)]) == 20:
                tmp += 2
            if tmp > 9:
                break
        return pts + tmp
    if scenario == "msgdropsinglefailure":
        pts = _join_points(lines, 15)
        fn = failed[0]
        pts += 15 if len(_grep(removed, fn)) >= 9 else 0
        return pts
    raise ValueError(scenario)
