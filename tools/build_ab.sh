# build a variant of libcapjwt.so with extra compile flags for ONE source
# (A/B measurement; load it with CAPJWT_LIB=...).
#   usage: tools/build_ab.sh NAME SRC "FLAGS"      SRC: a kernels/*.hip file name or jg_runtime.cpp
set -e
cd "$(dirname "$0")/../cap_amd/csrc"
name=$1; src=$2; flags=$3
mkdir -p build_ab/$name
base=$(basename $src)
if [ "$base" = "jg_runtime.cpp" ]; then
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $flags -x hip -c jg_runtime.cpp -o build_ab/$name/$base.o
else
  extra=""
  [ "$base" = "rsa.hip" ] && extra="-mllvm -pragma-unroll-threshold=500000"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $extra $flags -c kernels/$base -o build_ab/$name/$base.o
fi
objs=""
for o in build/*.hip.o build/jg_runtime.cpp.o; do [ "$(basename $o)" = "$base.o" ] || objs="$objs $o"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../ab_$name.so build_ab/$name/$base.o $objs
echo "built cap_amd/ab_$name.so"
