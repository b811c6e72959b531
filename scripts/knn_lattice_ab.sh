#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# worst case for the kNN paths: an exact lattice at rest (every row tied every step)
#   bash scripts/knn_lattice_ab.sh tree other   (build/lib_<name>; "tree" = in-tree lib)
for r in 1 2; do for n in "$@"; do lib=$PWD/build/lib_$n/libgymflock.so; [ "$n" = tree ] && lib=$PWD/gym-flock_amd/lib/libgymflock.so
for s in 20 200; do echo "lattice $n steps=$s $(GYMFLOCK_LIB=$lib LAYOUT=lattice KSTEPS=$s WARM=5 timeout -k 10 120 python scripts/knn_line.py 2>&1 | tail -1)"; done; done; done
