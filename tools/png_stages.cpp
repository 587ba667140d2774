// png_stages.cpp — design tool (not product code): times the PNG path of
// rt_main (rt_ppm_to_png: read the P3 file back, parse, filter, deflate,
// CRC, write) and rt_write_png alone on the same pixels, medians of N runs.
// Built against a png.cpp given on the command line, so two versions of the
// encoder can be timed side by side on one box:
//   clang++ -O3 -std=c++17 -DPNG_SRC='"path/png.cpp"' -I include \
//       -I raytracing-clj_amd/csrc tools/png_stages.cpp -lz -lpthread -o tools/bin/png_stages
//   tools/bin/png_stages scene.ppm out.png [runs=7]
#include PNG_SRC
#include <chrono>

namespace rtclj {
int set_error(int code, const std::string& msg) {
  std::fprintf(stderr, "error %d: %s\n", code, msg.c_str());
  return code;
}
void clear_error() {}
}  // namespace rtclj

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const int runs = argc > 3 ? std::atoi(argv[3]) : 7;
  std::vector<double> tot, wr;
  for (int r = 0; r < runs; ++r) {
    auto t = std::chrono::steady_clock::now();
    if (rt_ppm_to_png(argv[1], argv[2]) != 0) return 1;
    tot.push_back(ms_since(t));
  }
  // the pixels, parsed simply, for rt_write_png alone
  FILE* f = std::fopen(argv[1], "rb");
  int w = 0, h = 0, mx = 0;
  if (!f || std::fscanf(f, "P3 %d %d %d", &w, &h, &mx) != 3) return 1;
  std::vector<uint8_t> rgb(static_cast<size_t>(w) * h * 3);
  for (auto& v : rgb) {
    int x;
    if (std::fscanf(f, "%d", &x) != 1) return 1;
    v = static_cast<uint8_t>(x);
  }
  std::fclose(f);
  const std::string o2 = std::string(argv[2]) + ".direct.png";
  for (int r = 0; r < runs; ++r) {
    auto t = std::chrono::steady_clock::now();
    if (rt_write_png(o2.c_str(), rgb.data(), w, h) != 0) return 1;
    wr.push_back(ms_since(t));
  }
  std::sort(tot.begin(), tot.end());
  std::sort(wr.begin(), wr.end());
  std::printf("{\"ppm_to_png_ms\": %.3f, \"write_png_ms\": %.3f, \"parse_ms_est\": %.3f, \"threads\": %d, \"w\": %d, \"h\": %d}\n",
              tot[runs / 2], wr[runs / 2], tot[runs / 2] - wr[runs / 2], png_threads(), w, h);
  return 0;
}
