// Tile plan of the persistent halo conv (hconv3.hip), shared with the hconv dispatcher (hconv.hip).
#pragma once
#include "api.h"

namespace dcnn {

struct H3Plan {
  int HN;            // halo DMA instructions per wave and chunk (kernel instance)
  int TH, TW;        // output tile (16 x 16 pixels)
  int GY, GX;        // images per tile along y / x (> 1: small maps in the gutter layout)
  int IH, IW;        // image window of the tile (IH = TH unless gutter layout)
  int pitch;         // halo row pitch (pixels)
  int tx_tiles, tpi; // tiles per image row / per image group
  int splits, tiles_m, tiles_n;
};
bool hconv3_plan(int NB, int H, int W, int Cs, int N, int ntaps, H3Plan* pl);
bool hconv3_try(const HConvArgs& a, hipStream_t s);

}  // namespace dcnn
