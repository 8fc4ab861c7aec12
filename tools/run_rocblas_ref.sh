#!/bin/bash
# rocBLAS reference throughput on the C3 top-level shapes (comparison only, not the product)
set -e
hipcc -O3 --offload-arch=gfx950 tools/rocblas_ref.cpp -lrocblas -o /tmp/rbref
timeout -k 5 300 /tmp/rbref
