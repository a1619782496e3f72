#!/bin/bash
# SVGP A/B (tests, then interleaved bench lines) followed by a kernel trace of the in-tree library
set -o pipefail
OUT=${OUT:-svab} VARIANT=$VARIANT N=${N:-2} TESTS=${TESTS:-1} bash tools/gpu_svgp_ab.sh || exit $?
OUT=${OUT:-svab}_tr bash tools/gpu_svgp_trace.sh || exit $?
