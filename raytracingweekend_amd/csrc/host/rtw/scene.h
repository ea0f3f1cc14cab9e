// scene.h — scene container + the reference's scenes, and the host render API.
//
// `scene` keeps the accessors of the reference (Scene/scene.h:18-40):
// GetWorld, GetLights, GetCamera, GetRenderType, GetBackgroundType, Add.
// The concrete scenes restate Scene/scene.h:42-250 (light_sample,
// dielectric_scene, random_balls_scene, cornell_box_scene) plus Book 2's
// final scene (not in the reference; see scenes.cpp).
#pragma once
#include <memory>
#include <string>
#include <vector>
#include "camera.h"
#include "hittable_list.h"

enum class RenderType { Shaded, Normal };
enum class BackgroundType { Black, Gradient };

class scene {
public:
    scene() {}
    virtual ~scene() {}

    void Add(std::shared_ptr<hittable> h) { world.objects.push_back(h); }
    const hittable_list& GetWorld() const { return world; }
    std::shared_ptr<hittable_list> GetLights() const { return lights; }
    RenderType GetRenderType() const { return render_type; }
    BackgroundType GetBackgroundType() const { return background_type; }
    camera& GetCamera() { return cam; }
    const camera& GetCamera() const { return cam; }

protected:
    hittable_list world;
    std::shared_ptr<hittable_list> lights = std::make_shared<hittable_list>();
    camera cam;
    RenderType render_type = RenderType::Shaded;
    BackgroundType background_type = BackgroundType::Gradient;
};

class light_sample : public scene {
public:
    explicit light_sample(double aspect);
};
class dielectric_scene : public scene {
public:
    explicit dielectric_scene(double aspect);
};
class random_balls_scene : public scene {
public:
    explicit random_balls_scene(double aspect);
};
class cornell_box_scene : public scene {
public:
    explicit cornell_box_scene(double aspect);
};
class book2_final_scene : public scene {
public:
    explicit book2_final_scene(double aspect);
};
// Test scene for arbitrary nesting (transforms and media inside lists).
class nested_scene : public scene {
public:
    explicit nested_scene(double aspect, bool media = true);
};

// Builds a scene by name ("cornell_box", "random_balls", "dielectric",
// "light_sample", "book2_final", "nested", "nested_plain"); nullptr for an
// unknown name.
std::unique_ptr<scene> make_builtin_scene(const std::string& name, double aspect);

// Flatten the hittable graph of `sc` into a library-owned rtw_scene_desc
// (free with rtw_scene_desc_free).  Returns 0 or a negative rtw_status and
// sets rtw_last_error().  use_bvh: build device BVHs (world, and groups with
// more than a handful of primitives).
int rtw_flatten_scene(const scene& sc, int use_bvh, rtw_scene_desc** out);
