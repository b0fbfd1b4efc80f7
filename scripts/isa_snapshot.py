"""Device-assembly snapshot of every kernel translation unit, for refactors that must not
change the product's machine code (rejected experiments taken out of the
sources with the compiled kernels unchanged).

    python scripts/isa_snapshot.py OUTDIR [--csrc DIR]
    python scripts/isa_snapshot.py --compare DIR_A DIR_B

Writes OUTDIR/<tu>.s (hipcc --cuda-device-only -S with the library's flags) with the lines
that name source files or hold metadata dropped, then --compare lists the kernels whose
instruction text differs."""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as ge  # noqa: E402


def snapshot(out: str, csrc: str = ge.CSRC, jobs: int = 8) -> None:
    os.makedirs(out, exist_ok=True)
    tus = sorted(f for f in os.listdir(csrc) if f.endswith(".hip"))

    def one(tu):
        dst = os.path.join(out, tu[:-4] + ".s")
        subprocess.run([ge.HIPCC, *ge.tu_flags(tu), "--cuda-device-only", "-S", os.path.join(csrc, tu), "-o", dst],
                       check=True, capture_output=True)
        return tu

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for tu in ex.map(one, tus):
            print("snapshot", tu, flush=True)


def kernels(path: str) -> dict:
    """kernel symbol -> its instruction lines (comments, directives' paths and metadata dropped)."""
    out, cur = {}, None
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is None:
            continue
        s = line.split(";")[0].rstrip()
        if not s or s.startswith("\t.") or s.startswith("."):
            if s.startswith(".Lfunc_end"):
                cur = None
            continue
        out[cur].append(s)
    return out


def compare(a: str, b: str) -> int:
    bad = 0
    for f in sorted(os.listdir(a)):
        if not f.endswith(".s"):
            continue
        pb = os.path.join(b, f)
        if not os.path.exists(pb):
            print(f"{f}: missing in {b}")
            bad += 1
            continue
        ka, kb = kernels(os.path.join(a, f)), kernels(pb)
        for k in sorted(set(ka) | set(kb)):
            if k not in kb or k not in ka:
                print(f"{f}: {k[:80]} only in {'A' if k in ka else 'B'}")
                continue
            if ka[k] != kb[k]:
                bad += 1
                print(f"{f}: {k[:80]}: {len(ka[k])} vs {len(kb[k])} instructions differ")
    print("identical" if bad == 0 else f"{bad} differences")
    return bad


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?")
    ap.add_argument("--csrc", default=ge.CSRC)
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        sys.exit(1 if compare(*a.compare) else 0)
    snapshot(a.out, a.csrc)
