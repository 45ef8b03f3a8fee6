#!/usr/bin/env bash
# Builds the REFERENCE (nickmvincent/Surprise, Cython) out of tree, for golden-fixture
# generation in the CPU container only (tests/golden/make_golden.py).  Nothing built here
# is committed or shipped to the GPU box, and no reference source enters this repository:
# the sources are copied to a scratch directory outside the repo ($REF_BUILD, default
# /tmp/surprise_ref_build) and compiled there with the reference's own setup.py.
#
# One compatibility edit is applied to the scratch copy, never to /root/reference:
# NumPy 2's Cython declarations dropped `np.int_t`, used by three NON-hot-path modules
# (co_clustering.pyx, slope_one.pyx, similarities.pyx) that prediction_algorithms/__init__.py
# imports transitively; they are switched to `np.int64_t`.  matrix_factorization.pyx (the
# hot path) compiles unmodified.
set -euo pipefail
REF_SRC=${REF_SRC:-/root/reference}
REF_BUILD=${REF_BUILD:-/tmp/surprise_ref_build}
if [ -f "$REF_BUILD/.built" ]; then echo "$REF_BUILD"; exit 0; fi
rm -rf "$REF_BUILD"
mkdir -p "$REF_BUILD"
cp -r "$REF_SRC/surprise" "$REF_SRC/setup.py" "$REF_SRC/README.md" "$REF_SRC/requirements.txt" "$REF_BUILD/"
chmod -R u+w "$REF_BUILD"
for f in co_clustering slope_one; do
  sed -i 's/np\.int_t/np.int64_t/g' "$REF_BUILD/surprise/prediction_algorithms/$f.pyx"
done
sed -i 's/np\.int_t/np.int64_t/g' "$REF_BUILD/surprise/similarities.pyx"
( cd "$REF_BUILD" && python setup.py build_ext --inplace >build.log 2>&1 && python setup.py egg_info >>build.log 2>&1 )
touch "$REF_BUILD/.built"
echo "$REF_BUILD"
