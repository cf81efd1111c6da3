#!/bin/bash
# Kernel timeline of the download decode leg (descriptor copy kernel on the
# context's descriptor stream, mixed-row decode on the caller's stream).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/tr -o run -- \
  python3 bench.py --erase-pattern download --minimal --no-check --steps 50 --warmup 5 > $out/bench.json 2> $out/err.log || exit $?
python3 - $out <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/tr/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-150:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows[:60]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s/1e3:10.1f} {e/1e3:10.1f} {(e-s)/1e3:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:60]}")
PY
