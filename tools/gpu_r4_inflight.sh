#!/bin/bash
# (superseded by gpu_r4_bsort.sh, which runs the same sweep after its A/B)
bash "$(dirname "$0")/gpu_r4_bsort.sh"
