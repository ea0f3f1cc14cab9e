// validate.cpp — rtw_scene_upload's check of a caller-supplied scene desc
// (include/rtw_gpu.h): every count, index and pointer the kernels and the
// upload will follow is in range before anything is copied or launched.
// Host code only (no HIP), so the sanitizer build of the host library
// (tests/test_sanitizers.py) runs it under ASan / UBSan.
#include <cstdint>
#include <string>
#include <vector>
#include "rtw_host_util.h"

int validate_desc(const rtw_scene_desc* d) {
    if (!d) return rtw_fail(RTW_ERR_INVALID, "null scene desc");
    if (d->abi_version != RTW_ABI_VERSION) return rtw_fail(RTW_ERR_INVALID, "scene desc ABI version mismatch");
    if (d->n_entries < 0 || d->n_prims < 0 || d->n_materials < 0 || d->n_textures < 0 || d->n_lights < 0 ||
        d->n_bvh_nodes < 0 || d->n_bvh_items < 0 || d->n_visits < 0)
        return rtw_fail(RTW_ERR_INVALID, "negative array size in scene desc");
    if (d->n_entries > (1 << 20) - 1)  // the media walk packs entry indices in 20 bits (rtw_device.h)
        return rtw_fail(RTW_ERR_UNSUPPORTED, "more than 2^20 - 1 entries in scene desc");
    if ((d->n_entries && !d->entries) || (d->n_prims && !d->prims) || (d->n_materials && !d->materials) ||
        (d->n_textures && !d->textures) || (d->n_lights && !d->lights) || (d->n_bvh_nodes && !d->bvh_nodes) ||
        (d->n_bvh_items && !d->bvh_items) || (d->n_visits && !d->visits) ||
        (d->has_perlin && (!d->perlin_ranvec || !d->perlin_perm)))
        return rtw_fail(RTW_ERR_INVALID, "null array with a nonzero count in scene desc");
    for (int e = 0; e < d->n_entries; ++e) {
        const rtw_entry& E = d->entries[e];
        if (E.first_prim < 0 || E.n_prims <= 0 || (int64_t)E.first_prim + E.n_prims > d->n_prims)
            return rtw_fail(RTW_ERR_INVALID, "entry " + std::to_string(e) + ": prim range out of bounds");
        if (E.kind != RTW_ENTRY_GROUP && E.kind != RTW_ENTRY_MEDIUM)
            return rtw_fail(RTW_ERR_INVALID, "entry " + std::to_string(e) + ": bad kind");
        if (E.n_ops < 0 || E.n_ops > RTW_MAX_OPS) return rtw_fail(RTW_ERR_INVALID, "entry op count out of range");
        for (int k = 0; k < E.n_ops; ++k)
            if (E.op[k] != RTW_OP_TRANSLATE && E.op[k] != RTW_OP_ROTATE_Y && E.op[k] != RTW_OP_FLIP)
                return rtw_fail(RTW_ERR_INVALID, "entry " + std::to_string(e) + ": bad op type");
        if (E.n_outer_ops < 0 || E.n_outer_ops > E.n_ops || (E.kind != RTW_ENTRY_MEDIUM && E.n_outer_ops != 0))
            return rtw_fail(RTW_ERR_INVALID, "entry outer op count out of range");
        if (E.kind == RTW_ENTRY_MEDIUM && (E.phase_material < 0 || E.phase_material >= d->n_materials))
            return rtw_fail(RTW_ERR_INVALID, "medium phase material out of range");
        if (E.bvh_root >= d->n_bvh_nodes || E.bvh_root < -1)
            return rtw_fail(RTW_ERR_INVALID, "entry bvh root out of range");
        if (E.kind == RTW_ENTRY_MEDIUM && d->world_bvh_root >= 0)
            return rtw_fail(RTW_ERR_UNSUPPORTED, "a world BVH cannot hold media (list order matters for their draws)");
    }
    for (int p = 0; p < d->n_prims; ++p) {
        const rtw_prim& P = d->prims[p];
        if (P.type < RTW_PRIM_SPHERE || P.type > RTW_PRIM_RECT_YZ) return rtw_fail(RTW_ERR_INVALID, "bad prim type");
        if (P.material < 0 || P.material >= d->n_materials) return rtw_fail(RTW_ERR_INVALID, "prim material out of range");
        if (P.entry < -1 || P.entry >= d->n_entries) return rtw_fail(RTW_ERR_INVALID, "prim entry out of range");
    }
    // Every prim of an entry's range names that entry (hit_record reads the
    // winner's transforms and flips through prims[i].entry), and every prim
    // outside all ranges -- a light's own copy -- names none: traversal never
    // returns it, and a prim claimed by two ranges cannot name both.
    {
        std::vector<int> owner(d->n_prims, -1);
        for (int e = 0; e < d->n_entries; ++e) {
            const rtw_entry& E = d->entries[e];
            for (int i = E.first_prim; i < E.first_prim + E.n_prims; ++i) {
                if (owner[i] != -1)
                    return rtw_fail(RTW_ERR_INVALID, "prim " + std::to_string(i) + " belongs to entries " +
                                                         std::to_string(owner[i]) + " and " + std::to_string(e));
                owner[i] = e;
            }
        }
        for (int p = 0; p < d->n_prims; ++p)
            if (d->prims[p].entry != owner[p])
                return rtw_fail(RTW_ERR_INVALID, "prim " + std::to_string(p) + " names entry " +
                                                     std::to_string(d->prims[p].entry) + " but lies in entry " +
                                                     std::to_string(owner[p]) + "'s range");
    }
    for (int m = 0; m < d->n_materials; ++m) {
        const rtw_material& M = d->materials[m];
        const bool tex = M.type == RTW_MAT_LAMBERTIAN || M.type == RTW_MAT_DIFFUSE_LIGHT || M.type == RTW_MAT_ISOTROPIC;
        if (M.type < RTW_MAT_LAMBERTIAN || M.type > RTW_MAT_ISOTROPIC) return rtw_fail(RTW_ERR_INVALID, "bad material type");
        if (tex && (M.texture < 0 || M.texture >= d->n_textures)) return rtw_fail(RTW_ERR_INVALID, "material texture out of range");
    }
    for (int t = 0; t < d->n_textures; ++t) {
        const rtw_texture& T = d->textures[t];
        if (T.type == RTW_TEX_NOISE && !d->has_perlin) return rtw_fail(RTW_ERR_INVALID, "noise texture without perlin tables");
        if (T.type == RTW_TEX_CHECKER && (T.odd < 0 || T.odd >= d->n_textures || T.even < 0 || T.even >= d->n_textures))
            return rtw_fail(RTW_ERR_INVALID, "checker child out of range");
    }
    for (int l = 0; l < d->n_lights; ++l) {
        const rtw_light& L = d->lights[l];
        if (L.kind < RTW_LIGHT_DEFAULT || L.kind > RTW_LIGHT_SPHERE) return rtw_fail(RTW_ERR_INVALID, "bad light kind");
        if (L.kind != RTW_LIGHT_DEFAULT && (L.prim < 0 || L.prim >= d->n_prims))
            return rtw_fail(RTW_ERR_INVALID, "light prim out of range");
        if ((L.kind == RTW_LIGHT_XZ_RECT && d->prims[L.prim].type != RTW_PRIM_RECT_XZ) ||
            (L.kind == RTW_LIGHT_SPHERE && d->prims[L.prim].type != RTW_PRIM_SPHERE &&
             d->prims[L.prim].type != RTW_PRIM_MOVING_SPHERE))
            return rtw_fail(RTW_ERR_INVALID, "light " + std::to_string(l) + ": its prim is not of the light's shape");
    }
    if (d->n_visits < 0 || (d->n_visits > 0 && !d->visits)) return rtw_fail(RTW_ERR_INVALID, "bad visit program");
    for (int k = 0; k < d->n_visits; ++k) {
        const int v = d->visits[k];
        if (v < 0 || (v & ~(RTW_VISIT_ENTRY | RTW_VISIT_REPLAY)) || (v & RTW_VISIT_ENTRY) >= d->n_entries)
            return rtw_fail(RTW_ERR_INVALID, "visit " + std::to_string(k) + " out of range");
    }
    if (d->n_visits > 0 && d->world_bvh_root >= 0)
        return rtw_fail(RTW_ERR_UNSUPPORTED, "a visit program walks the list: no world BVH with it");
    if (d->world_bvh_root >= d->n_bvh_nodes || d->world_bvh_root < -1)
        return rtw_fail(RTW_ERR_INVALID, "world bvh root out of range");
    for (int k = 0; k < d->n_bvh_nodes; ++k) {
        const rtw_bvh_node& N = d->bvh_nodes[k];
        if (N.count < 0) return rtw_fail(RTW_ERR_INVALID, "bvh node out of range");
        if (N.count > 0 ? (N.left < 0 || (int64_t)N.left + N.count > d->n_bvh_items)
                        : (N.left < 0 || N.left >= d->n_bvh_nodes || N.right < 0 || N.right >= d->n_bvh_nodes))
            return rtw_fail(RTW_ERR_INVALID, "bvh node out of range");
    }
    // Each BVH is a tree (no node reached twice, so walks terminate and the
    // upload's depth count is finite) whose leaf items lie in its domain:
    // prims of the entry's own range (group BVH) or entry indices (world).
    {
        std::vector<int> seen(d->n_bvh_nodes, 0);
        auto walk = [&](int root, int lo, int hi, const char* what, bool group_items) -> int {
            std::vector<int> todo{root};
            while (!todo.empty()) {
                const int n = todo.back();
                todo.pop_back();
                if (seen[n]++) return rtw_fail(RTW_ERR_INVALID, std::string(what) + " BVH is not a tree");
                const rtw_bvh_node& N = d->bvh_nodes[n];
                if (N.count == 0) {
                    todo.push_back(N.left);
                    todo.push_back(N.right);
                    continue;
                }
                for (int k = N.left; k < N.left + N.count; ++k) {
                    int it = d->bvh_items[k], span = 1;
                    if (!group_items && it < 0)
                        return rtw_fail(RTW_ERR_INVALID, std::string(what) + " BVH item out of range");
                    if (group_items && it >= 0 && (it & RTW_ITEM_BOX)) {  // a box: six rects in box order
                        it &= RTW_ITEM_INDEX;
                        span = 6;
                        static const int kBoxTypes[6] = {RTW_PRIM_RECT_XY, RTW_PRIM_RECT_XY, RTW_PRIM_RECT_XZ,
                                                         RTW_PRIM_RECT_XZ, RTW_PRIM_RECT_YZ, RTW_PRIM_RECT_YZ};
                        if (it >= lo && (int64_t)it + 6 <= hi)
                            for (int j = 0; j < 6; ++j)
                                if (d->prims[it + j].type != kBoxTypes[j])
                                    return rtw_fail(RTW_ERR_INVALID, "box item " + std::to_string(k) +
                                                                         ": its prims are not a box's six rects");
                    }
                    if (it < lo || (int64_t)it + span > hi)
                        return rtw_fail(RTW_ERR_INVALID, std::string(what) + " BVH item out of range");
                }
            }
            return RTW_OK;
        };
        for (int e = 0; e < d->n_entries; ++e) {
            const rtw_entry& E = d->entries[e];
            if (E.bvh_root < 0) continue;
            if (int rc = walk(E.bvh_root, E.first_prim, E.first_prim + E.n_prims, "group", true)) return rc;
        }
        if (d->world_bvh_root >= 0)
            if (int rc = walk(d->world_bvh_root, 0, d->n_entries, "world", false)) return rc;
    }
    return RTW_OK;
}
