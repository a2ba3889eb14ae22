// examples/box_demo.cpp — the reference application's scene (an open box of five mirror-ish
// walls lit by two point lights, 1000x1000, focal 500; RaytracingEngine.cpp:223-290 without
// the OBJ model whose box.obj is absent) built with the unchanged reference API, rendered on
// the MI355X, tonemapped with all seven operators on the device and written as PPM files.
//
//   g++ -std=c++20 -ffp-contract=off -I raytracingengine_amd/api -I include
//       examples/box_demo.cpp -L raytracingengine_amd -lrtamd_cpp -lrtamd
#include "Image.h"
#include "Light.h"
#include "Math.h"
#include "Scene.h"
#include "Shape.h"

#include <chrono>
#include <iostream>
#include <string>

int main(int argc, char** argv) {
    const size_t side = argc > 1 ? std::stoul(argv[1]) : 1000;
    const int aa = argc > 2 ? std::stoi(argv[2]) : 1;
    Camera camera(Vec3(0, 0, -25), side / 2.0, side, side, 0, 200);
    camera.antiAliasingAmount = aa;
    Scene scene(camera);
    scene.SetCountRays(true);

    struct Wall { Vec3 dir, color; };
    const Wall walls[] = {{Vec3(0, 0, -1), Vec3(1, 1, 1)}, {Vec3(1, 0, 0), Vec3(0, 1, 0)},
                          {Vec3(-1, 0, 0), Vec3(0, 0, 1)}, {Vec3(0, 1, 0), Vec3(1, 1, 1)},
                          {Vec3(0, -1, 0), Vec3(1, 1, 1)}};
    for (const Wall& w : walls) {
        Material m;
        m.color = w.color;
        m.specular = 0.01;
        m.shininess = 0.128;
        m.refractiveIndex = 1.5;
        Plane wall(w.dir * -15.0, w.dir, m);
        scene.AddPlane(wall);
    }
    Light key(Vec3(0, 0, -5), Vec3(1, 1, 1), 150), fill(Vec3(-2, 2, -5), Vec3(1, 1, 1), 150);
    scene.AddLight(key);
    scene.AddLight(fill);

    const auto t0 = std::chrono::steady_clock::now();
    const std::vector<Vec3> hdr = scene.RenderImage();
    const auto t1 = std::chrono::steady_clock::now();
    const rt_stats st = scene.LastStats();
    std::cout << "render " << std::chrono::duration<double, std::milli>(t1 - t0).count()
              << " ms (" << st.trace_rays << " trace + " << st.shadow_rays << " shadow rays)\n";

    const char* names[] = {"simple", "reinhard_simple", "reinhard_extended",
                           "reinhard_extended_luminance", "reinhard_jodie", "uncharted2", "aces"};
    const auto all = rtamd::tonemapAll(hdr);
    for (size_t i = 0; i < all.size(); ++i)
        writePPM(std::string(names[i]) + ".ppm", all[i], side, side);
    return 0;
}
