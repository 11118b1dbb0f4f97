#!/bin/bash
# Phase-B/C balance of the tile BFS with partial-tile masks: 1000^2 VGA global kernel time and digest for
# a list of environment settings (ENVS: ';'-separated, each a space-separated list of VAR=value).
set -o pipefail
O=gpurun_out/${TAG:-vga_env}
mkdir -p $O
if [ -n "$LIBV" ] && [ "$LIBV" != "none" ]; then export DMX_LIB=depthmapx_amd/_lib_ab/$LIBV/libdmx.so; fi
IFS=';' read -ra SETS <<< "${ENVS:-DMX_VGA_BEXT=4}"
for e in "${SETS[@]}"; do
  env $e timeout -k 10 200 python -u scripts/probe_vga_time.py --reps 1 >> $O/ab.log 2>> $O/ab.err || exit 1
done
cut -c1-300 $O/ab.log
