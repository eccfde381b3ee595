/* Include-path shim for <lora_phy/ChirpGenerator.hpp>: genChirp (float) is declared in
 * lora_mi355x_phy.hpp and exported by liblora_mi355x.so. */
#pragma once
#include "../../lora_mi355x_phy.hpp"
