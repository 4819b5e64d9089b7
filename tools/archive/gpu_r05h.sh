#!/bin/bash
# round 5, pass h: full GPU suite + smoke + bench at HEAD, then the step A/B against the r05a library
set -u
R=$PWD
bash tools/gpu_suite.sh r05h || exit 1
bash tools/gpu_lib_ab.sh r05h/ab 3 || exit 1
