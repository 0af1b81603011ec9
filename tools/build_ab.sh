# build a variant of libcapjwt.so with extra compile flags for some sources
# (A/B measurement; load it with CAPJWT_LIB=..., or copy it over
# cap_amd/libcapjwt.so on the GPU box for the host extension's paths).
#   usage: tools/build_ab.sh NAME SRC[,SRC...] "FLAGS"      SRC: kernels/*.hip file names or jg_runtime.cpp
set -e
cd "$(dirname "$0")/../cap_amd/csrc"
name=$1; srcs=$2; flags=$3
mkdir -p build_ab/$name
mine=""
for src in ${srcs//,/ }; do
  base=$(basename $src)
  mine="$mine $base.o"
  if [ "$base" = "jg_runtime.cpp" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $flags -x hip -c jg_runtime.cpp -o build_ab/$name/$base.o
  else
    extra=""
    [ "$base" = "rsa.hip" ] && extra="-mllvm -pragma-unroll-threshold=500000"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $extra $flags -c kernels/$base -o build_ab/$name/$base.o &
  fi
done
wait
objs=""
for o in build/*.hip.o build/jg_runtime.cpp.o; do
  b=$(basename $o)
  case " $mine " in *" $b "*) objs="$objs build_ab/$name/$b" ;; *) objs="$objs $o" ;; esac
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../ab_$name.so $objs
echo "built cap_amd/ab_$name.so"
