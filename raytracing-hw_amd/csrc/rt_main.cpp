// rt_main.cpp — drop-in CLI for the reference's `solution` (src/main.cpp:22-60, run.sh:2):
//   rt_solution input.gltf width height samples [output.ppm]
// Same positional arguments, same default output name, same terminate-with-message
// behaviour on errors (std::runtime_error), rendering through librt_hw_amd on every GPU of
// the node (rt_render_frame: one row-block shard per device, finished on its GPU and gathered
// device-to-device onto GPU 0; RT_GPUS=n uses devices 0..n-1).
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <iostream>
#include <iomanip>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rt_hw.h"

static void check(int rc) {
    if (rc != RT_OK) throw std::runtime_error(rt_last_error());
}

static int int_arg(const char *s) { return std::stoi(std::string(s).substr(0, std::string(s).find(' '))); }

int main(int argc, char *argv[]) {
    if (argc < 5 || argc > 6)
        throw std::runtime_error("Invalid arguments - " + std::to_string(argc) + " (expected: 5)");
    std::string input = argv[1];
    int width = int_arg(argv[2]), height = int_arg(argv[3]), samples = int_arg(argv[4]);
    std::string output = argc == 6 ? argv[5] : "output.ppm";

    std::cout << "Loading scene." << std::endl;
    auto t0 = std::chrono::steady_clock::now();
    rt_scene *scene = nullptr;
    check(rt_scene_load_gltf(input.c_str(), width, height, samples, &scene));
    auto t1 = std::chrono::steady_clock::now();
    std::cout << "Scene loaded: " << std::setprecision(2) << std::chrono::duration<double>(t1 - t0).count()
              << " seconds." << std::endl;
    std::cout << std::setprecision(6) << "Rendering scene." << std::endl;
    const char *g = std::getenv("RT_GPUS");
    const int n_gpus = g ? std::atoi(g) : 0;   // 0: every visible device
    rt_params p{};
    p.spp = samples;
    p.row_block = 8;
    rt_stats st{};
    // every shard finished to 8 bits on its GPU and gathered device-to-device onto GPU 0
    std::vector<uint8_t> rgb((size_t)width * height * 3);
    check(rt_render_frame(scene, &p, n_gpus, nullptr, rgb.data(), nullptr, &st));
    double total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::cout << "      " << total << " seconds (" << total * 1000 << " ms) elapsed; render " << st.render_ms
              << " ms on " << st.devices << " MI355X." << std::endl;
    check(rt_write_ppm(output.c_str(), rgb.data(), width, height));
    std::cout << "Frame drawn into " << output << std::endl;
    rt_scene_free(scene);
    return 0;
}
