#!/usr/bin/env bash
# A/B of single-matrix (cant-like) cold/warm kernel times under rocprofv3,
# one library per run (SPMV_HIP_LIB; "tree" = the in-tree library).
# usage: tools/ab_single.sh NAME=LIB[,NAME=LIB...] [cant_single.py args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
libs=$1; shift
IFS=, read -ra pairs <<< "$libs"
for p in "${pairs[@]}"; do
  name=${p%%=*}; lib=${p#*=}
  d=gpurun_out/ab_single_$name
  rm -rf "$d"
  if [ "$lib" = tree ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run -- python3 tools/cant_single.py --json "$d.json" "$@" > "$d.log" 2>&1
  else
    SPMV_HIP_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run -- python3 tools/cant_single.py --json "$d.json" "$@" > "$d.log" 2>&1
  fi
  rc=$?
  echo "=== $name ($lib) exit $rc"
  [ $rc -ne 0 ] && { tail -20 "$d.log"; exit $rc; }
  timeout -k 10 120 python tools/cant_single.py --json "$d.json" --attach "$d" > /dev/null || exit 1
  python - "$d.json" <<'PY'
import json, sys
o = json.load(open(sys.argv[1]))
for k, v in list(o["formats"].items()) + [("stream_probe", o["stream_probe"])]:
    print(f"  {k:40s} cold {v.get('cold_ms')} ms ({v.get('cold_GBs')} GB/s, frac {v.get('cold_frac')})  warm {v.get('warm_ms')} ms  "
          f"parity {v.get('parity_ok', '-')}  {v.get('kernels', '')}")
PY
done
