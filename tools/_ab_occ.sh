#!/bin/bash
# Occupancy A/B of the integrate: register targets (compile-time variants) and grid sizes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
ROUNDS=${ROUNDS:-2} bash tools/_ab.sh "X=1" "SEMTSDF_LIB=$R/build/var_wpe5.so" "SEMTSDF_LIB=$R/build/var_wpe3.so" "SEMTSDF_GRID_PER_CU=2" "SEMTSDF_GRID_PER_CU=3"
