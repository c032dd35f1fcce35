#!/usr/bin/env bash
# Compaction with one returning atomic per wave and no block barriers (variant 155 = 154 |
# VAR_WAVE_ATOMIC) against the default block-aggregated compaction (154), in one process
set -u
cd "$(dirname "$0")/.."
timeout -k 10 300 python tools/ab_variants.py --variants 154,155 --rounds 5 --frames 40 --scene cornell > gpurun_out/waveatomic_cornell.json && \
timeout -k 10 300 python tools/ab_variants.py --variants 154,155 --rounds 3 --frames 40 --scene cornell_glass_test > gpurun_out/waveatomic_glass.json && \
python3 -c "
import json
for f in ('cornell','glass'):
    d=json.load(open('gpurun_out/waveatomic_%s.json'%f)); print(f, {k:v['ms_per_frame_median'] for k,v in d['results'].items()})"
