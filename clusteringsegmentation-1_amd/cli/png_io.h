// png_io.h -- PNG read/write for the ClusteringSegmentation CLI (the
// reference reads and writes images with OpenCV imread/imwrite,
// ClusteringSegmentationMain.cpp:94, :114; OpenCV is not in this image, so
// the CLI carries its own codec over the system zlib).
//
// Reading follows imread(..., CV_LOAD_IMAGE_COLOR): every image becomes 8-bit
// BGR (alpha dropped, grey replicated, palette expanded, 16-bit samples
// reduced to their high byte).  Non-interlaced PNGs of every colour type and
// bit depth; Adam7-interlaced files are rejected with a message.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace dqcli {

struct Image {
  uint32_t width = 0, height = 0;
  std::vector<uint8_t> bgr;   // height rows of 3 * width bytes (B, G, R)
};

// false (with a reason in *err) when the file is missing or not a supported PNG
bool read_png_bgr(const std::string& path, Image* img, std::string* err);
// 8-bit RGB PNG from BGR rows (imwrite of a CV_8UC3 Mat)
bool write_png_bgr(const std::string& path, const Image& img, std::string* err);

}  // namespace dqcli
