// .npz writer for training rows (reference trainingwrite.cpp:566-587 layout).
#pragma once
#include <cstdint>
#include <string>

namespace kc {

// Rows are host arrays in the coffee_selfplay_drain_rows layout.
void writeNpz(const std::string& path, int n, int X, int Y, const uint8_t* bin, const float* glob,
              const int16_t* pol, const float* gt, const int8_t* val);

}  // namespace kc
