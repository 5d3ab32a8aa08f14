#!/bin/bash
# Build the A/B variants of the score-scan kernel timed by tools/variant_bench.py
# (one library per variant, same sources, different -D knobs).
set -e
B="python diversity-recommendations_amd/build_native.py --jobs 8"
$B --variant base -D DR_NUT=2 -D DR_STAGE_BYTES=16384 -D DR_RING=4 -D DR_PRIO=0 -D DR_APIPE=0 -D DR_FLUSH_GAP=100000 -D DR_PREPASS=0
$B --variant nut2 -D DR_NUT=2
$B --variant prio -D DR_PRIO=1
$B --variant noapipe -D DR_APIPE=0
$B --variant pre -D DR_PREPASS=1
$B --variant ring3 -D DR_RING=3
$B --variant gap32 -D DR_FLUSH_GAP=32
$B --variant gap256 -D DR_FLUSH_GAP=256
