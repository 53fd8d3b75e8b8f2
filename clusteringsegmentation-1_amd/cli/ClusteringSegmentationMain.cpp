// ClusteringSegmentation IMAGE ?TAGS_IMAGE? -- the reference's command line
// (ClusteringSegmentation/ClusteringSegmentationMain.cpp:48-120), driving the
// MI355X DivQuant path through the drop-in headers (include/quant_util.h,
// include/DivQuantHeader.h) and the C ABI (include/dq_hip.h).
//
// In scope (the hot path of SURVEY.md section 8): the argv contract, image
// read/write, the BGR24 -> packed-pixel conversion (Vec3BToUID), the
// full-frame 125-colour map + 4x4 block histograms of genHistogramsForBlocks
// (ClusteringSegmentation.cpp:365-576, with its two dump images), and
// quant_recurse over the image (allPixelsUnique = 0, as every app call site,
// ClusteringSegmentation.cpp:1803).  The TAGS_IMAGE written here tags every
// pixel with its DivQuant cluster: the pixel's index in the deduplicated
// colortable, as a colour (PixelToVec3b).  Out of scope: the SRM
// segmentation, the superpixel containment tree and the region merge loop of
// clusteringCombine (:124-383) -- sequential union-find / graph heuristics
// on OpenCV types, not this data-parallel path.
//
// DQ_TAGS_K (default 256): the cluster count of the whole-image quant_recurse.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <unistd.h>

#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/DivQuantHeader.h"
#include "../../include/dq_hip.h"
#include "../../include/quant_util.h"
#include "png_io.h"

using namespace std;

namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    cerr << "HIP error in " << what << ": " << hipGetErrorString(e) << endl;
    exit(1);
  }
}

// PixelToVec3b (superpixels/OpenCVUtil.h:53-59) of a frame of packed pixels,
// on the GPU, into an image of width x height.
bool unpack_to_image(int dev, const uint32_t* d_px, uint32_t width, uint32_t height, dqcli::Image* img) {
  uint8_t* d_bgr = nullptr;
  hip_check(hipMalloc((void**)&d_bgr, (size_t)width * height * 3), "hipMalloc");
  if (dq_hip_unpack_bgr24_dev(dev, d_px, width, height, 3 * width, d_bgr, nullptr) != 0) return false;
  img->width = width;
  img->height = height;
  img->bgr.resize((size_t)width * height * 3);
  hip_check(hipDeviceSynchronize(), "unpack");
  hip_check(hipMemcpy(img->bgr.data(), d_bgr, img->bgr.size(), hipMemcpyDeviceToHost), "hipMemcpy");
  hip_check(hipFree(d_bgr), "hipFree");
  return true;
}

bool write_image(const string& name, const dqcli::Image& img) {
  string err;
  if (!dqcli::write_png_bgr(name, img, &err)) {
    cerr << "could not write \"" << name << "\": " << err << endl;
    return false;
  }
  cout << "wrote " << name << endl;
  return true;
}

// The in-scope part of clusteringCombine on the GPU.
bool clusteringCombine(const dqcli::Image& input, dqcli::Image* result) {
  const int dev = 0;
  const uint32_t width = input.width, height = input.height, n = width * height;
  // Constant for block of 4x4 based map (ClusteringSegmentationMain.cpp:138-149)
  const uint32_t superpixelDim = 4;
  const uint32_t blockWidth = (width + superpixelDim - 1) / superpixelDim;
  const uint32_t blockHeight = (height + superpixelDim - 1) / superpixelDim;
  assert(blockWidth * superpixelDim >= width && blockHeight * superpixelDim >= height);

  // The Mat's BGR rows -> packed 0x00RRGGBB pixels (Vec3BToUID), on the GPU
  uint8_t* d_bgr = nullptr;
  uint32_t *d_px = nullptr, *d_quant = nullptr, *d_mode = nullptr;
  hip_check(hipSetDevice(dev), "hipSetDevice");
  hip_check(hipMalloc((void**)&d_bgr, input.bgr.size()), "hipMalloc");
  hip_check(hipMalloc((void**)&d_px, (size_t)n * 4), "hipMalloc");
  hip_check(hipMalloc((void**)&d_quant, (size_t)n * 4), "hipMalloc");
  hip_check(hipMalloc((void**)&d_mode, (size_t)blockWidth * blockHeight * 4), "hipMalloc");
  hip_check(hipMemcpy(d_bgr, input.bgr.data(), input.bgr.size(), hipMemcpyHostToDevice), "hipMemcpy");
  if (dq_hip_pack_bgr24_dev(dev, d_bgr, width, height, 3 * width, d_px, nullptr) != 0) return false;

  // genHistogramsForBlocks (ClusteringSegmentation.cpp:365-576): the frame
  // mapped onto getSubdividedColors, then the most frequent colour of every
  // 4x4 block; both dumped as the reference does (:410-412, :564-568)
  uint32_t palette[125];
  dq_subdivided_colors(palette);
  if (dq_hip_block_hist_dev(dev, d_px, width, height, palette, 125, superpixelDim, blockWidth, blockHeight,
                            d_quant, d_mode, nullptr, nullptr, nullptr, nullptr) != 0)
    return false;
  dqcli::Image img;
  if (!unpack_to_image(dev, d_quant, width, height, &img) || !write_image("block_quant_full_output.png", img))
    return false;
  if (!unpack_to_image(dev, d_mode, blockWidth, blockHeight, &img) || !write_image("block_quant_output.png", img))
    return false;

  // quant_recurse over the image through its C signature (quant_util.h)
  vector<uint32_t> in(n), out(n);
  hip_check(hipMemcpy(in.data(), d_px, (size_t)n * 4, hipMemcpyDeviceToHost), "hipMemcpy");
  const char* ks = getenv("DQ_TAGS_K");
  uint32_t k = ks && *ks ? (uint32_t)atoi(ks) : 256u;
  if (k == 0) k = 1;
  vector<uint32_t> colortable(k);
  const uint32_t kreq = k;
  quant_recurse(n, in.data(), out.data(), &k, colortable.data(), 0);
  cout << "quant_recurse K=" << kreq << " -> " << k << " colours" << endl;

  // tags: a pixel's index in the (deduplicated) colortable
  unordered_map<uint32_t, uint32_t> tag_of;
  for (uint32_t i = 0; i < k; ++i) tag_of.emplace(colortable[i], i);
  vector<uint32_t> tags(n);
  for (uint32_t i = 0; i < n; ++i) {
    auto it = tag_of.find(out[i]);
    if (it == tag_of.end()) {
      cerr << "mapped colour 0x" << hex << out[i] << dec << " is not in the colortable" << endl;
      return false;
    }
    tags[i] = it->second;
  }
  hip_check(hipMemcpy(d_quant, tags.data(), (size_t)n * 4, hipMemcpyHostToDevice), "hipMemcpy");
  if (!unpack_to_image(dev, d_quant, width, height, result)) return false;
  for (void* p : {(void*)d_bgr, (void*)d_px, (void*)d_quant, (void*)d_mode}) hip_check(hipFree(p), "hipFree");
  return true;
}

}  // namespace

int main(int argc, const char** argv) {
  const char* inputImgFilename = NULL;
  const char* outputTagsImgFilename = NULL;

  if (argc == 2) {
    inputImgFilename = argv[1];
    // Default to "outtags.png"
    outputTagsImgFilename = "outtags.png";
    // A path with a directory: cd there and read the file by its base name
    // (the reference does this for Xcode's profiling tools, :59-81).
    const char* slash = strrchr(inputImgFilename, '/');
    if (slash) {
      string dirname(inputImgFilename, (size_t)(slash - inputImgFilename));
      inputImgFilename = slash + 1;
      cout << "cd \"" << dirname << "\"" << endl;
      if (chdir(dirname.c_str()) != 0) {
        cerr << "could not cd to \"" << dirname << "\"" << endl;
        exit(1);
      }
    }
  } else if (argc != 3) {
    cerr << "usage : " << argv[0] << " IMAGE ?TAGS_IMAGE?" << endl;
    cerr << "  (MI355X DivQuant path: block histograms + DivQuant cluster tags; the SRM / superpixel" << endl;
    cerr << "   stages of the reference pipeline are not part of this build)" << endl;
    exit(1);
  } else {
    inputImgFilename = argv[1];
    outputTagsImgFilename = argv[2];
  }

  cout << "read \"" << inputImgFilename << "\"" << endl;

  dqcli::Image inputImg;
  string err;
  if (!dqcli::read_png_bgr(inputImgFilename, &inputImg, &err)) {
    cerr << "could not read \"" << inputImgFilename << "\" as image data (" << err << ")" << endl;
    exit(1);
  }
  if (inputImg.height == 0 || inputImg.width == 0) {
    cerr << "invalid size " << inputImg.width << "x" << inputImg.height << " for image data" << endl;
    exit(1);
  }
  if (dq_hip_device_count() < 1) {
    cerr << "no HIP device: the DivQuant path runs on the GPU only" << endl;
    exit(1);
  }

  dqcli::Image resultImg;
  const bool worked = clusteringCombine(inputImg, &resultImg);
  if (!worked) {
    cerr << "cluster combine operation failed " << endl;
    exit(1);
  }
  if (!dqcli::write_png_bgr(outputTagsImgFilename, resultImg, &err)) {
    cerr << "could not write \"" << outputTagsImgFilename << "\": " << err << endl;
    exit(1);
  }
  cout << "wrote " << outputTagsImgFilename << endl;
  exit(0);
}
