#!/bin/bash
# Experimental builds of libecg.so with extra compile flags, for A/B runs that
# load a library by path (tools/crc_libs.py).  usage: tools/build_exp.sh NAME "FLAGS"
set -e
cd "$(dirname "$0")/../daos_amd/csrc"
name=$1
flags=$2
make -s -j8 OUT=../../build/exp/$name OBJ=../../build/exp/$name/obj EXP_HIPFLAGS="$flags"
