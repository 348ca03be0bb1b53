// Segment table of the ragged pack kernel (csrc/detection/pack_images.hip), shared with the host packer that builds it
// (csrc/bindings/fastcall.cpp map_pack).
#pragma once
#include <cstdint>

namespace tm_amd {

enum PackMode : int16_t { kPackCopy = 0, kPackZero = 1, kPackXyxyToXywh = 2 };

struct PackSeg {
  const void* src;  // nullptr for kPackZero
  void* dst;
  int32_t n;        // elements (kPackCopy / kPackZero) or box rows (kPackXyxyToXywh)
  int16_t esize;    // bytes per element (4 or 8 for boxes)
  int16_t mode;
};

// Copy / zero / convert every segment: ceil(n / 128) launches of one block per segment (the table travels as kernel
// arguments), on the current stream of `device`.
void pack_segments(const PackSeg* segs, int n, int device);

}  // namespace tm_amd
