#!/bin/bash
# round 5, pass ac: full GPU suite + smoke + bench at HEAD
set -u
bash tools/gpu_suite.sh r05ac || exit 1
