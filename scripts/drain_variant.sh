#!/bin/bash
# Drain-kernel A/B helper: libgossip_amd.<tag>.so = the product objects (build/, from `make lib`)
# with pview_drain.hip recompiled from <src> and extra flags.  Loaded with GSP_LIB_VARIANT=<tag>
# (scripts/ab_drain.sh).
#   bash scripts/drain_variant.sh <tag> [<pview_drain.hip source>] [hipcc flags...]
set -euo pipefail
cd "$(dirname "$0")/.."
TAG=${1:?usage: $0 <tag> [src] [flags...]}
SRC=${2:-gossip_protocol_amd/csrc/pview_drain.hip}
shift $(( $# >= 2 ? 2 : 1 ))
mkdir -p "build/dv-$TAG"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Iinclude -Igossip_protocol_amd/csrc \
    -I/opt/rocm/include "$@" -c "$SRC" -o "build/dv-$TAG/pview_drain.hip.o"
objs=$(ls build/*.o | grep -v '/pview_drain.hip.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -o "gossip_protocol_amd/libgossip_amd.$TAG.so" $objs \
    "build/dv-$TAG/pview_drain.hip.o" -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "gossip_protocol_amd/libgossip_amd.$TAG.so"
