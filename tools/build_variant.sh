#!/bin/bash
# Experiment library for same-box A/B: recompile the named sources with extra flags, link them with the product
# objects of every other source -> deep-rawburst-sr_amd/libdbsr_hip_<name>.so (load with DBSR_HIP_LIB=...).
#   bash tools/build_variant.sh <name> "<flags>" conv_fuse [conv2d ...]
set -e
name=$1; flags=$2; shift 2
PKG=deep-rawburst-sr_amd
make -s -j8 >/dev/null
mkdir -p $PKG/build/v_$name
objs=""
for o in $PKG/build/*.o; do
  b=$(basename $o .o)
  if [[ " $* " == *" $b "* ]]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Wall -Wno-unused-function $flags \
        -c $PKG/csrc/$b.hip -o $PKG/build/v_$name/$b.o
    objs="$objs $PKG/build/v_$name/$b.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $PKG/libdbsr_hip_$name.so $objs
echo "built $PKG/libdbsr_hip_$name.so"
