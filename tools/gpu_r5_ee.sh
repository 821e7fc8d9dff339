#!/bin/bash
# round 5: rocprofv3 kernel trace of one 10 h bench step on the final kernels (bench.py now exits normally
# at world 1, so the profiler's exit-time flush runs)
NAME=r5_e2e_prof TO=480 bash tools/gpu_prof.sh
