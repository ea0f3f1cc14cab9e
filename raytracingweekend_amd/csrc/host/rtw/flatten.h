// flatten.h — the drop-in seam for the reference's own scene class.
//
// The reference's render loop reads its scene only through five accessors
// (Scene/scene.h:24-31): GetWorld() (const hittable_list&), GetLights()
// (shared_ptr<hittable_list>), GetCamera() (camera&, non-const),
// GetRenderType() and GetBackgroundType().  rtw_flatten() takes ANY class with
// those accessors -- the reference's unchanged `scene` and its subclasses
// included, compiled against this directory's hittable / material / camera
// headers -- and flattens it into an rtw_scene_desc for rtw_scene_upload.
// This header does not include scene.h, so it can sit next to the reference's
// own Scene/scene.h, which defines `scene`, RenderType and BackgroundType
// itself.
//
// The enums are passed by value: RenderType {Shaded, Normal} and
// BackgroundType {Black, Gradient} (Scene/scene.h:6-16) are 0 / 1 in both the
// reference and rtw_gpu.h (RTW_RENDER_SHADED / _NORMAL, RTW_BG_BLACK /
// _GRADIENT).
#pragma once
#include "camera.h"
#include "hittable_list.h"
#include "rtw_gpu.h"

// The flattener proper (flatten.cpp).  lights may be null (no light list).
int rtw_flatten_world(const hittable_list& world, const hittable_list* lights, const camera& cam, int render_type,
                      int background, int use_bvh, rtw_scene_desc** out);

template <class Scene>
int rtw_flatten(Scene& sc, int use_bvh, rtw_scene_desc** out) {
    const auto lights = sc.GetLights();
    return rtw_flatten_world(sc.GetWorld(), lights.get(), sc.GetCamera(), static_cast<int>(sc.GetRenderType()),
                             static_cast<int>(sc.GetBackgroundType()), use_bvh, out);
}
