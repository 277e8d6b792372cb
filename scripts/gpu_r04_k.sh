#!/bin/bash
# TopN diagnosis: host stacks + GC pauses, then kernel stats.
set -o pipefail
bash scripts/gpu_r04_i.sh && bash scripts/gpu_r04_j.sh
