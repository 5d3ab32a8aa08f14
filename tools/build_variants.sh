#!/bin/bash
# Build the A/B variant of the score scan that the product keeps a knob for
# (one library per variant, same sources, a different -D): the d = 128 stage
# size, 64 KB against the product's 72 KB (profiles/r06/stage_fetch/: time
# and PMC FETCH side by side). Planner choices are runtime knobs instead
# (dr_set_plan_knob; tools/variant_bench.py tags "product@knob=value").
set -e
B="python diversity-recommendations_amd/build_native.py --jobs 8"
$B --variant stage64 -D DR_STAGE_BYTES_WIDE=65536
