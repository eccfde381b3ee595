#!/bin/bash
# Build an A/B variant of the library: tools/build_variant.sh NAME "-DFLAG ..."
# -> lora-sdr-lightweight-standalone-library-_amd/lora_phy_amd/lib/variants/NAME.so
# (select it at run time with LORA_MI355X_LIB=<path>).
set -e
cd "$(dirname "$0")/../lora-sdr-lightweight-standalone-library-_amd"
mkdir -p lora_phy_amd/lib/variants
make -s ARCH=gfx950 OUT=lora_phy_amd/lib/variants/$1.so EXTRA="$2" lora_phy_amd/lib/variants/$1.so
