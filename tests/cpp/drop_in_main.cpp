// TEST PROGRAM: the reference's main.cpp flow (main.cpp:368-397) on the MI355X path through the
// C++ drop-in header -- what INTEGRATION.md asks a maintainer to change, compiled and linked the
// way a host program would (g++, -I include, -l simplepath_hip).  tests/test_drop_in.py runs it.
//
//   drop_in_main <scene.sp | -> [--samples N] [--integrator NAME] [--bvh 0|1] [--size W H] [--output FILE]
//                [--from-desc]
#include "simplepath_amd.hpp"

#include <cstdlib>
#include <cstring>
#include <iostream>
#include <iterator>
#include <string>

int main(int argc, char** argv)
{
    if (argc < 2) {
        std::cerr << "usage: " << argv[0] << " scene.sp [--samples N] [--integrator NAME] [--bvh 0|1] [--size W H]"
                  << " [--output FILE] [--from-desc]\n";
        return EXIT_FAILURE;
    }
    std::string    file_path = argv[1], output, integrator_name;
    unsigned       num_pixel_samples = 8;
    int            bvh = 0, width = 0, height = 0;
    bool           from_desc = false;
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--samples" && i + 1 < argc) num_pixel_samples = static_cast<unsigned>(std::atoi(argv[++i]));
        else if (a == "--integrator" && i + 1 < argc) integrator_name = argv[++i];
        else if (a == "--bvh" && i + 1 < argc) bvh = std::atoi(argv[++i]);
        else if (a == "--size" && i + 2 < argc) { width = std::atoi(argv[++i]); height = std::atoi(argv[++i]); }
        else if (a == "--output" && i + 1 < argc) output = argv[++i];
        else if (a == "--from-desc") from_desc = true;
        else {
            std::cerr << "unknown argument " << a << '\n';
            return EXIT_FAILURE;
        }
    }
    try {
        sp_amd::IntegratorType integrator_type = sp_amd::IntegratorType::NotSpecified;
        if (!integrator_name.empty()) integrator_type = sp_amd::string_to_integrator_type(integrator_name);
        sp_amd::Scene scene;
        if (file_path == "-") {
            const std::string text{ std::istreambuf_iterator<char>(std::cin), std::istreambuf_iterator<char>() };
            scene = sp_amd::parse_scene_text(text);
        } else {
            scene = sp_amd::parse_scene_file(file_path);
        }
        if (width > 0) scene.set_resolution(width, height);
        if (from_desc) { // a host-built scene handed over without re-parsing
            sp_scene_desc d{};
            sp_amd::check(sp_scene_get_desc(scene.handle(), &d));
            sp_amd::Scene copy = sp_amd::Scene::from_desc(d);
            scene              = std::move(copy);
        }
        if (!output.empty()) scene.output_file_name = output;
        // main.cpp:387-392
        if (integrator_type == sp_amd::IntegratorType::NotSpecified) integrator_type = scene.integrator_type;
        if (integrator_type == sp_amd::IntegratorType::NotSpecified) integrator_type = sp_amd::IntegratorType::DirectLighting;
        const auto integrator = sp_amd::create_integrator(integrator_type, scene.image_width, scene.image_height,
                                                          scene.russian_roulette_depth, scene.max_depth);
        scene.upload(0, bvh);
        sp_amd::render(*integrator, 1, num_pixel_samples, scene);
        std::cout << "wrote " << scene.output_file_name << " (" << scene.image_width << "x" << scene.image_height
                  << ", " << num_pixel_samples << " spp)\n";
    } catch (const sp_amd::ParsingException& e) {
        std::cerr << "ParsingException: " << e.what() << '\n';
        return 2;
    } catch (const std::exception& e) {
        std::cerr << e.what() << '\n';
        return EXIT_FAILURE;
    }
    return EXIT_SUCCESS;
}
