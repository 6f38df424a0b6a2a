#!/bin/bash
# variant libraries for timing experiments: tools/jx_build.sh NAME -DMACRO ...
name=$1; shift
python -m geomesa_amd.build --out=$PWD/geomesa_amd/lib/$name.so "$@" > /dev/null
