#!/bin/bash
# Build the clock-probe variant of libglx (-DGLX_CLOCK_PROBE) into abtree/probe, a copy of the
# package + bench.py, so that the shipped library stays stamp-free (scripts/clock_probe.py).
set -e
cd "$(dirname "$0")/.."
rm -rf abtree/probe && mkdir -p abtree/probe
cp -r bench.py oracle include abtree/probe/
mkdir -p abtree/probe/convex-optimization_amd
cp -r convex-optimization_amd/csrc convex-optimization_amd/glx convex-optimization_amd/Makefile convex-optimization_amd/gl_*.py abtree/probe/convex-optimization_amd/
rm -rf abtree/probe/convex-optimization_amd/glx/__pycache__ abtree/probe/convex-optimization_amd/glx/libglx.so
make -C abtree/probe/convex-optimization_amd -j8 \
  CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -I../include -Icsrc -DGLX_CLOCK_PROBE" > /dev/null
ls -la abtree/probe/convex-optimization_amd/glx/libglx.so
