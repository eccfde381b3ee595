/* Include-path shim: a caller written against the reference's <lora_phy/phy.hpp> legacy
 * helpers compiles unchanged with -I<repo>/include/compat and links -llora_mi355x. */
#pragma once
#include "../../lora_mi355x_phy.hpp"
