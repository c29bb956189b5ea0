#!/bin/bash
# Diagnostic gather-structure kernels (scripts/diag_gather_shapes.hip) -> scripts/ab/libdiag_gather.so
set -e
cd "$(dirname "$0")/.."
mkdir -p scripts/ab
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared scripts/diag_gather_shapes.hip -o scripts/ab/libdiag_gather.so
