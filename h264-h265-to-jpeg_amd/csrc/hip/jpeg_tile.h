// Layout of one 256-block tile of the JPEG symbol stream (K4c symbol form -> K4e / K5b / K5d);
// the host sizes the per-frame region from H2J_JTILE_BYTES (include/h2j_gpu.h).
#pragma once
#include "h2j_gpu.h"

constexpr int kJSymMax = H2J_JSYM_MAX;                   // AC symbols per block: <= 63 + 3 ZRL + EOB
constexpr size_t kJCntOff = static_cast<size_t>(kJSymMax) * 256 * 4;  // uint8 symbol count per block
constexpr size_t kJDcOff = kJCntOff + 256;               // int16 quantised DC per block
constexpr size_t kJTileBytes = H2J_JTILE_BYTES;
static_assert(kJDcOff + 512 == kJTileBytes, "JPEG tile layout");
