#!/bin/bash
# Same-box ABAB of two builds on one GPU box (the pattern behind every profiles/r04*_ab_*
# file): the tree's libraries against a directory built by tools/ab_build.sh.
#   tools/gpu_ab.sh LIB_DIR TAG [REPEATS] -- command args...
# e.g. tools/gpu_ab.sh ab_old r05a 2 -- tools/lg_bench.py --pairs 2048 --iters 2
# Runs `python -u <command>` for the tree, then through tools/ab_run.py --lib-dir LIB_DIR,
# REPEATS times (default 2), each under its own time limit, and prints every JSON line of
# every run; stops at the first failure.
set -u
LIB="$1"; TAG="$2"; shift 2
REP=2
if [ "${1:-}" != "--" ]; then REP="$1"; shift; fi
[ "${1:-}" = "--" ] && shift
mkdir -p gpurun_out
for ((k = 0; k < REP; ++k)); do
  for arm in tree "$LIB"; do
    if [ "$arm" = tree ]; then pre=""; else pre="tools/ab_run.py --lib-dir $LIB"; fi
    log="gpurun_out/${TAG}_$(basename "$arm")_$k.log"
    timeout -k 10 300 python -u $pre "$@" > "$log" 2>&1 || { echo "$arm failed"; tail -5 "$log"; exit 1; }
    grep '^{' "$log" | cut -c1-400 | sed "s|^|$arm |"
  done
done
