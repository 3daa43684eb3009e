// SceneConfig -> host scene graph, restating packages/ray-tracer/src/scene_config.rs.
//
// Deserialisation follows serde's externally tagged enums: a config value is a
// table with exactly one key naming the variant.  `textures`, `materials` and
// `instances` are accepted both in the current `[[id, {Kind: {...}}], ...]`
// sequence form (scene_config.rs:387-400) and in the legacy TOML table form
// `[textures.<id>.<Kind>]` used by spheres.toml / earth.toml,
// keeping document order; the older index-based schema of triangles.toml is
// normalised onto the current one first (normalize_legacy).
#include "scene_config.hpp"

#include <algorithm>
#include <cmath>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>

namespace nrt {

namespace {

[[noreturn]] void fail(const std::string& msg) { throw std::runtime_error(msg); }

std::string read_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) fail("No such file or directory (os error 2): " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

double as_f64(const Value& v, const char* what) {
    if (!v.is_number()) fail(std::string("invalid type for `") + what + "`: expected f64");
    return v.number();
}

uint64_t as_usize(const Value& v, const char* what) {
    if (v.kind != Value::Int || v.i < 0) fail(std::string("invalid type for `") + what + "`: expected usize");
    return (uint64_t)v.i;
}

uint32_t as_u32(const Value& v, const char* what) {
    if (v.kind != Value::Int || v.i < 0 || v.i > 0xFFFFFFFFll) fail(std::string("invalid type for `") + what + "`: expected u32");
    return (uint32_t)v.i;
}

V3 as_dvec3(const Value& v, const char* what) {
    if (v.kind != Value::Array || v.arr.size() != 3)
        fail(std::string("invalid value for `") + what + "`: expected a sequence of 3 numbers");
    return v3(as_f64(v.arr[0], what), as_f64(v.arr[1], what), as_f64(v.arr[2], what));
}

std::string as_str(const Value& v, const char* what) {
    if (v.kind != Value::String) fail(std::string("invalid type for `") + what + "`: expected a string");
    return v.s;
}

// Field access helpers: required / optional (null or missing = None).
const Value& req(const Value& t, const char* key, const char* ctx) {
    const Value* v = t.get(key);
    if (!v) fail(std::string("missing field `") + key + "` in " + ctx);
    return *v;
}
const Value* opt(const Value& t, const char* key) {
    const Value* v = t.get(key);
    if (!v || v->is_null()) return nullptr;
    return v;
}

// serde externally tagged enum: {Variant: {fields}}
std::pair<std::string, const Value*> variant(const Value& v, const char* ctx) {
    if (v.kind != Value::Table || v.tab.size() != 1)
        fail(std::string("invalid ") + ctx + ": expected a table with a single variant key");
    const Value& body = v.tab[0].second;
    if (body.kind != Value::Table) fail(std::string("invalid ") + ctx + " '" + v.tab[0].first + "': expected a table");
    return {v.tab[0].first, &body};
}

// Vec<(Box<str>, T)>: sequence of 2-element sequences, or (legacy) a table.
std::vector<std::pair<std::string, const Value*>> id_list(const Value* v, const char* ctx) {
    std::vector<std::pair<std::string, const Value*>> out;
    if (!v || v->is_null()) return out;
    if (v->kind == Value::Array) {
        for (const Value& e : v->arr) {
            if (e.kind != Value::Array || e.arr.size() != 2 || e.arr[0].kind != Value::String)
                fail(std::string("invalid ") + ctx + " entry: expected [id, config]");
            out.emplace_back(e.arr[0].s, &e.arr[1]);
        }
        return out;
    }
    if (v->kind == Value::Table) {
        for (const auto& kv : v->tab) out.emplace_back(kv.first, &kv.second);
        return out;
    }
    fail(std::string("invalid type for `") + ctx + "`: expected a sequence");
}

CameraConfig parse_camera_config(const Value& t) {
    if (t.kind != Value::Table) fail("invalid type for `camera`: expected a table");
    CameraConfig c;
    if (auto v = opt(t, "width")) { c.has_width = true; c.width = as_usize(*v, "width"); }
    if (auto v = opt(t, "height")) { c.has_height = true; c.height = as_usize(*v, "height"); }
    if (auto v = opt(t, "aspect_ratio")) { c.has_aspect_ratio = true; c.aspect_ratio = as_f64(*v, "aspect_ratio"); }
    if (auto v = opt(t, "background_color")) { c.has_background_color = true; c.background_color = as_dvec3(*v, "background_color"); }
    if (auto v = opt(t, "look_at")) { c.has_look_at = true; c.look_at = as_dvec3(*v, "look_at"); }
    if (auto v = opt(t, "look_from")) { c.has_look_from = true; c.look_from = as_dvec3(*v, "look_from"); }
    if (auto v = opt(t, "view_up")) { c.has_view_up = true; c.view_up = as_dvec3(*v, "view_up"); }
    if (auto v = opt(t, "focal_length")) { c.has_focal_length = true; c.focal_length = as_f64(*v, "focal_length"); }
    if (auto v = opt(t, "field_of_view")) { c.has_field_of_view = true; c.field_of_view = as_f64(*v, "field_of_view"); }
    if (auto v = opt(t, "defocus_angle")) { c.has_defocus_angle = true; c.defocus_angle = as_f64(*v, "defocus_angle"); }
    if (auto v = opt(t, "focus_distance")) { c.has_focus_distance = true; c.focus_distance = as_f64(*v, "focus_distance"); }
    if (auto v = opt(t, "samples_per_pixel")) { c.has_samples_per_pixel = true; c.samples_per_pixel = as_usize(*v, "samples_per_pixel"); }
    if (auto v = opt(t, "ray_max_bounces")) { c.has_ray_max_bounces = true; c.ray_max_bounces = as_usize(*v, "ray_max_bounces"); }
    return c;
}

using TextureMap = std::map<std::string, TexturePtr>;
using MaterialMap = std::map<std::string, MaterialPtr>;
using InstanceMap = std::map<std::string, ObjectPtr>;

// TextureConfig::try_make_texture (scene_config.rs:52-123)
TexturePtr make_texture(const Value& cfg, const TextureMap& textures) {
    auto [kind, body] = variant(cfg, "texture config");
    auto t = std::make_shared<Texture>();
    if (kind == "SolidColor") {
        t->kind = Texture::Solid;
        t->color = as_dvec3(req(*body, "color", "SolidColor"), "color");
    } else if (kind == "Image") {
        const std::string path = as_str(req(*body, "path", "Image"), "path");
        DecodedImage img = decode_image_file(path);
        t->kind = Texture::Image;
        t->width = img.width;
        t->height = img.height;
        t->texels = std::make_shared<std::vector<float>>(std::move(img.rgb));
    } else if (kind == "Checker") {
        t->kind = Texture::Checker;
        auto even = std::make_shared<Texture>();  // CheckerBuilder defaults (checker.rs:53-59)
        even->color = v3(1, 1, 1);
        auto odd = std::make_shared<Texture>();
        odd->color = v3(0, 0, 0);
        t->even = even;
        t->odd = odd;
        t->scale = 0.5;
        if (auto v = opt(*body, "even")) {
            auto it = textures.find(as_str(*v, "even"));
            if (it == textures.end()) fail("invalid texture index");
            t->even = it->second;
        }
        if (auto v = opt(*body, "odd")) {
            auto it = textures.find(as_str(*v, "odd"));
            if (it == textures.end()) fail("invalid texture index");
            t->odd = it->second;
        }
        if (auto v = opt(*body, "scale")) t->scale = as_f64(*v, "scale");
    } else if (kind == "Marble") {
        // MarbleBuilder::build (marble.rs:46-60): Fbm(seed), 7 octaves, frequency
        t->kind = Texture::Marble;
        if (auto v = opt(*body, "seed")) t->fbm.seed = as_u32(*v, "seed");
        if (auto v = opt(*body, "frequency")) t->fbm.frequency = as_f64(*v, "frequency");
        t->fbm.octaves = MARBLE_OCTAVES;
    } else if (kind == "Noise") {
        // PerlinRidgedNoiseBuilder::build (noise.rs:79-101): octaves default 1, then
        // Fbm::set_octaves clamps to [1, 32]
        t->kind = Texture::Noise;
        if (auto v = opt(*body, "seed")) t->fbm.seed = as_u32(*v, "seed");
        if (auto v = opt(*body, "frequency")) t->fbm.frequency = as_f64(*v, "frequency");
        if (auto v = opt(*body, "lacunarity")) t->fbm.lacunarity = as_f64(*v, "lacunarity");
        if (auto v = opt(*body, "persistence")) t->fbm.persistence = as_f64(*v, "persistence");
        uint64_t oct = 1;
        if (auto v = opt(*body, "octaves")) oct = as_usize(*v, "octaves");
        t->fbm.octaves = fbm_octaves(oct);
    } else {
        fail("unknown variant `" + kind + "` for TextureConfig");
    }
    return t;
}

TexturePtr get_texture(const Value* id, const TextureMap& textures, const TexturePtr& fallback) {
    if (!id) return fallback;
    const std::string s = as_str(*id, "texture");
    auto it = textures.find(s);
    if (it == textures.end()) fail("invalid texture id: '" + s + "'");
    return it->second;
}

// MaterialConfig::try_make_material (scene_config.rs:162-198)
MaterialPtr make_material(const Value& cfg, const TextureMap& textures, const TexturePtr& texture_fallback) {
    auto [kind, body] = variant(cfg, "material config");
    auto m = std::make_shared<Material>();
    if (kind == "Dielectric") {
        m->kind = Material::Dielectric;
        m->refraction_index = as_f64(req(*body, "refraction_index", "Dielectric"), "refraction_index");
    } else if (kind == "DiffuseLight") {
        m->kind = Material::DiffuseLight;
        m->intensity = as_f64(req(*body, "intensity", "DiffuseLight"), "intensity");
        m->texture = get_texture(opt(*body, "texture"), textures, texture_fallback);
    } else if (kind == "Lambertian") {
        m->kind = Material::Lambertian;
        m->texture = get_texture(opt(*body, "texture"), textures, texture_fallback);
    } else if (kind == "Metal") {
        m->kind = Material::Metal;
        m->fuzz = as_f64(req(*body, "fuzz", "Metal"), "fuzz");
        m->texture = get_texture(opt(*body, "texture"), textures, texture_fallback);
    } else {
        fail("unknown variant `" + kind + "` for MaterialConfig");
    }
    return m;
}

MaterialPtr get_material(const Value* id, const MaterialMap& materials, const MaterialPtr& fallback) {
    if (!id) return fallback;
    const std::string s = as_str(*id, "material");
    auto it = materials.find(s);
    if (it == materials.end()) fail("invalid material id: '" + s + "'");
    return it->second;
}

// The legacy scene schema of scenes/triangles.toml:22-189: `textures`
// and `materials` are arrays of variant tables referenced by integer index and the
// objects sit in `objects`.  It maps onto the current schema with ids "0", "1", ...
// -- the scene `nr-ray-tracer create triangles` now writes with named ids
// (create/triangles.rs:10-86).  Other documents are returned unchanged.  Opt-in
// (NRT_LOAD_LEGACY_SCHEMA): the reference's SceneConfig rejects the file (serde expects
// (id, config) pairs) and ignores an unknown `objects` key of a current-schema document.
Value legacy_refs(const Value& v) {
    Value out = v;
    if (v.kind == Value::Table) {
        for (auto& kv : out.tab) {
            const std::string& k = kv.first;
            if ((k == "material" || k == "texture" || k == "even" || k == "odd") && kv.second.kind == Value::Int) {
                Value id = Value::make(Value::String);
                id.s = std::to_string(kv.second.i);
                kv.second = id;
            } else {
                kv.second = legacy_refs(kv.second);
            }
        }
    } else if (v.kind == Value::Array) {
        for (auto& e : out.arr) e = legacy_refs(e);
    }
    return out;
}

Value normalize_legacy(const Value& doc) {
    if (doc.kind != Value::Table || !doc.get("objects") || doc.get("scene")) return doc;
    Value out = Value::make(Value::Table);
    for (const auto& [k, v] : doc.tab) {
        if (k == "objects") {
            out.tab.emplace_back("scene", legacy_refs(v));
        } else if ((k == "textures" || k == "materials") && v.kind == Value::Array &&
                   std::all_of(v.arr.begin(), v.arr.end(), [](const Value& e) { return e.kind == Value::Table; })) {
            Value list = Value::make(Value::Array);
            for (size_t i = 0; i < v.arr.size(); ++i) {
                Value pair = Value::make(Value::Array);
                Value id = Value::make(Value::String);
                id.s = std::to_string(i);
                pair.arr.push_back(id);
                pair.arr.push_back(legacy_refs(v.arr[i]));
                list.arr.push_back(pair);
            }
            out.tab.emplace_back(k, list);
        } else {
            out.tab.emplace_back(k, v);
        }
    }
    return out;
}

struct Builder {
    int depth = 0;
    bool legacy = false;  // accept the legacy index schema of scenes/triangles.toml (opt-in)

    // SceneConfig::try_build_aux (scene_config.rs:410-473)
    LoadedScene build_aux(const Value& doc, const MaterialPtr* material_fallback_in, const CameraConfig* cli) {
        if (doc.kind != Value::Table) fail("invalid scene file: expected a table");
        const Value& camera_v = req(doc, "camera", "SceneConfig");
        CameraConfig camera = parse_camera_config(camera_v);
        if (cli) camera.merge_with(*cli);

        TextureMap textures;
        for (auto& [id, cfg] : id_list(doc.get("textures"), "textures")) textures[id] = make_texture(*cfg, textures);

        TexturePtr texture_fallback;
        if (auto v = opt(doc, "texture_fallback")) {
            texture_fallback = make_texture(*v, textures);
        } else {
            texture_fallback = std::make_shared<Texture>();
            texture_fallback->kind = Texture::Solid;
            texture_fallback->color = 0.5 * v3(1, 1, 1);
        }

        MaterialMap materials;
        for (auto& [id, cfg] : id_list(doc.get("materials"), "materials"))
            materials[id] = make_material(*cfg, textures, texture_fallback);

        // `material_fallback.unwrap_or(<expr>)` evaluates <expr> eagerly, so the
        // file's own fallback is built (and may fail) even when a parent one exists.
        MaterialPtr own_fallback;
        if (auto v = opt(doc, "material_fallback")) {
            own_fallback = make_material(*v, textures, texture_fallback);
        } else {
            own_fallback = std::make_shared<Material>();
            own_fallback->kind = Material::Lambertian;
            own_fallback->texture = texture_fallback;
        }
        const MaterialPtr material_fallback = material_fallback_in ? *material_fallback_in : own_fallback;

        InstanceMap instances;
        for (auto& [id, cfg] : id_list(doc.get("instances"), "instances"))
            instances[id] = make_object(*cfg, instances, materials, material_fallback);

        std::vector<ObjectPtr> objects;
        if (const Value* sc = doc.get("scene"); sc && !sc->is_null()) {
            if (sc->kind != Value::Array) fail("invalid type for `scene`: expected a sequence");
            for (const Value& o : sc->arr) objects.push_back(make_object(o, instances, materials, material_fallback));
        }

        CameraBuilder cb;
        camera.try_update(cb);
        LoadedScene out;
        out.camera = camera_build(cb);
        out.objects = make_bvh(objects);
        return out;
    }

    // ObjectConfig::try_make_object (scene_config.rs:277-381)
    ObjectPtr make_object(const Value& cfg, const InstanceMap& instances, const MaterialMap& materials,
                          const MaterialPtr& fallback) {
        auto [kind, body] = variant(cfg, "object config");
        const Value& b = *body;
        if (kind == "Quad" || kind == "Triangle") {
            MaterialPtr m = get_material(opt(b, "material"), materials, fallback);
            return make_plane(kind == "Quad" ? Object::Quad : Object::Triangle, as_dvec3(req(b, "point", "Quad"), "point"),
                              as_dvec3(req(b, "u", "Quad"), "u"), as_dvec3(req(b, "v", "Quad"), "v"), m);
        }
        if (kind == "Sphere") {
            MaterialPtr m = get_material(opt(b, "material"), materials, fallback);
            return make_sphere(as_dvec3(req(b, "center", "Sphere"), "center"), as_f64(req(b, "radius", "Sphere"), "radius"), m);
        }
        if (kind == "Group") {
            MaterialPtr m = get_material(opt(b, "material"), materials, fallback);
            const Value& list = req(b, "objects", "Group");
            if (list.kind != Value::Array) fail("invalid type for `objects`: expected a sequence");
            std::vector<ObjectPtr> group;
            for (const Value& o : list.arr) group.push_back(make_object(o, instances, materials, m));
            return make_bvh(group);
        }
        if (kind == "Scene") {
            MaterialPtr m = get_material(opt(b, "material"), materials, fallback);
            const std::string path = as_str(req(b, "path", "Scene"), "path");
            if (++depth > 64) fail("nested Scene depth exceeds 64 (recursive scene file?)");
            LoadedScene child = build_aux(load_doc(path, legacy), &m, nullptr);
            --depth;
            return child.objects;
        }
        if (kind == "Ref") {
            const std::string id = as_str(req(b, "id", "Ref"), "id");
            auto it = instances.find(id);
            if (it == instances.end()) fail("invalid object id");
            return it->second;
        }
        const std::string kname = kind;
        auto child = [&]() { return make_object(req(b, "object", kname.c_str()), instances, materials, fallback); };
        if (kind == "RotateX") { double a = as_f64(req(b, "angle", "RotateX"), "angle"); return make_rotate(child(), v3(1, 0, 0), a); }
        if (kind == "RotateY") { double a = as_f64(req(b, "angle", "RotateY"), "angle"); return make_rotate(child(), v3(0, 1, 0), a); }
        if (kind == "RotateZ") { double a = as_f64(req(b, "angle", "RotateZ"), "angle"); return make_rotate(child(), v3(0, 0, 1), a); }
        if (kind == "ScaleU") {
            double f = as_f64(req(b, "factor", "ScaleU"), "factor");
            return make_scale(child(), f * v3(1, 1, 1));
        }
        if (kind == "ScaleV") { V3 s = as_dvec3(req(b, "scale", "ScaleV"), "scale"); return make_scale(child(), s); }
        if (kind == "Translate") { V3 o = as_dvec3(req(b, "offset", "Translate"), "offset"); return make_translate(child(), o); }
        fail("unknown variant `" + kind + "` for ObjectConfig");
    }

    // SceneConfig::try_load_scene (scene_config.rs:475-492): format by extension; the legacy
    // schema is mapped onto the current one only on request (the reference itself rejects it)
    static Value load_doc(const std::string& path, bool legacy) {
        const size_t dot = path.find_last_of('.');
        const size_t slash = path.find_last_of('/');
        const std::string ext = (dot == std::string::npos || (slash != std::string::npos && dot < slash)) ? "" : path.substr(dot + 1);
        Value doc;
        if (ext == "json") doc = parse_json(read_file(path));
        else if (ext == "toml") doc = parse_toml(read_file(path));
        else fail("invalid scene file format!");
        return legacy ? normalize_legacy(doc) : doc;
    }
};

}  // namespace

void CameraConfig::merge_with(const CameraConfig& o) {
    if (o.has_background_color) { has_background_color = true; background_color = o.background_color; }
    if (o.has_width) { has_width = true; width = o.width; }
    if (o.has_height) { has_height = true; height = o.height; }
    if (o.has_aspect_ratio) { has_aspect_ratio = true; aspect_ratio = o.aspect_ratio; }
    if (o.has_field_of_view) { has_field_of_view = true; field_of_view = o.field_of_view; }
    if (o.has_focus_distance) { has_focus_distance = true; focus_distance = o.focus_distance; }
    if (o.has_defocus_angle) { has_defocus_angle = true; defocus_angle = o.defocus_angle; }
    if (o.has_samples_per_pixel) { has_samples_per_pixel = true; samples_per_pixel = o.samples_per_pixel; }
    if (o.has_ray_max_bounces) { has_ray_max_bounces = true; ray_max_bounces = o.ray_max_bounces; }
    if (o.has_view_up) { has_view_up = true; view_up = o.view_up; }
    if (o.has_look_at) { has_look_at = true; look_at = o.look_at; }
    if (o.has_look_from) { has_look_from = true; look_from = o.look_from; }
    // focal_length is parsed but never merged (cli.rs:229, absent from 316-355)
}

void CameraConfig::try_update(CameraBuilder& b) const {
    // CameraConfig::get_size (cli.rs:273-312)
    const int key = (has_width ? 4 : 0) | (has_height ? 2 : 0) | (has_aspect_ratio ? 1 : 0);
    switch (key) {
        case 0: break;
        case 6: b.width = width; b.height = height; break;
        case 5: {  // ImageSize::from_width_and_aspect_ratio (image.rs:26-32)
            double h = (double)width / aspect_ratio;
            uint64_t hh = (h != h || h <= 0) ? 0 : (h >= 18446744073709551615.0 ? UINT64_MAX : (uint64_t)h);
            b.width = width; b.height = hh < 1 ? 1 : hh;
            break;
        }
        case 3: {
            double w = (double)height * aspect_ratio;
            uint64_t ww = (w != w || w <= 0) ? 0 : (w >= 18446744073709551615.0 ? UINT64_MAX : (uint64_t)w);
            b.width = ww < 1 ? 1 : ww; b.height = height;
            break;
        }
        case 4: fail("When '-W' or '--width' are specified, one of '-H', '--height', '-R', '--aspect-ratio' must be specified too.");
        case 2: fail("When '-H' or '--height' are specified, one of '-W', '--width', '-R', '--aspect-ratio' must be specified too.");
        case 1: fail("When '-R' or '--aspect-ratio' are specified, one of '-W', '--width', '-H', '--height' must be specified too.");
        default: fail("When '-R,' or '--aspect-ratio' are specified, '-W' or '--width' and '-H' or '--height' are mutually exclusive.");
    }
    if (has_background_color) b.background_color = background_color;
    if (has_field_of_view) b.field_of_view = (field_of_view * M_PI) / 180.0;
    if (has_focus_distance) b.focus_dist = focus_distance;
    if (has_defocus_angle) b.defocus_angle = (defocus_angle * M_PI) / 180.0;
    if (has_samples_per_pixel) b.samples_per_pixel = samples_per_pixel;
    if (has_ray_max_bounces) b.ray_max_bounces = ray_max_bounces;
    if (has_view_up) b.view_up = view_up;
    if (has_look_at) b.look_at = look_at;
    if (has_look_from) b.look_from = look_from;
}

LoadedScene load_scene_file(const std::string& path, const CameraConfig* cli, bool legacy_schema) {
    Builder b;
    b.legacy = legacy_schema;
    Value doc = Builder::load_doc(path, legacy_schema);
    return b.build_aux(doc, nullptr, cli);
}

}  // namespace nrt
