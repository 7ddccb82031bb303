#!/bin/bash
# quick GPU iteration: parity tests then phase profile
tools/gpu_step.sh pytest_gpu 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider || exit $?
tools/gpu_step.sh phase 300 python tools/phase_prof.py ${1:-256}
