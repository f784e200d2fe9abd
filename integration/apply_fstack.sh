#!/bin/sh
# Wire libespgpu into an F-Stack checkout (INTEGRATION.md sections 1-4):
#   integration/apply_fstack.sh <f-stack root> [--dry-run]
# copies the kernel-domain driver, the newbus glue and the host-domain shim
# into lib/ and applies fstack-ipsec-gpu.patch (lib/Makefile: the FF_IPSEC
# source lists made to compile and link, FF_IPSEC_GPU sources and include
# path; kproc_create / fpu_kern_thread / zfree glue; lib/ff_api.symlist;
# lib/ff_init.c GPU context; lib/ff_dpdk_if.c main_loop poll).  Build F-Stack
# with FF_IPSEC=1 FF_IPSEC_GPU=1 ESPGPU_ROOT=<this repo>.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=${1:?usage: apply_fstack.sh <f-stack root> [--dry-run]}
if [ "$2" = "--dry-run" ]; then
  patch -p1 --dry-run -d "$ROOT" < "$HERE/fstack-ipsec-gpu.patch"
  exit 0
fi
patch -p1 -d "$ROOT" < "$HERE/fstack-ipsec-gpu.patch"
cp "$HERE/ff_gpucrypto.c" "$HERE/ff_gpucrypto_host.c" "$HERE/ff_newbus.c" "$ROOT/lib/"
