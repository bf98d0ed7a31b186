# Build compile-time variants of the native library for tools/abvariant.py:
#   bash tools/build_variants.sh name:-DFLAG[,-DFLAG2] ...
# -> tools/variants/<name>/libingot_gpu.so (parse.hip rebuilt with the flags,
# the other objects taken from the in-tree build).
set -e
cd "$(dirname "$0")/.."
python -m ingot_amd.build
for v in "$@"; do
    n=${v%%:*}; f=${v#*:}
    mkdir -p tools/build/$n tools/variants/$n
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
        -Iinclude ${f//,/ } -c ingot_amd/csrc/parse.hip -o tools/build/$n/parse.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/$n/libingot_gpu.so \
        tools/build/$n/parse.o $(ls ingot_amd/build/*.o | grep -v parse.hip.o)
done
