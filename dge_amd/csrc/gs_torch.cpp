// gs_torch.cpp — compiled torch binding of the per-view render() path (round 6).
//
// dge_amd/_C.py binds the C ABI (include/gs_raster.h) through ctypes: every call builds ctypes structs
// attribute by attribute, checks and converts each tensor in Python and crosses into the library through
// libffi — ~25 us of host time before a training render's first kernel is enqueued (DGE's loop idles the
// GPU for all of it after each of its per-view host syncs, threestudio/systems/DGE.py:198-213).  This module
// does the same work for the calls DGE's loop makes per view — the raw-parameter forward's two halves
// (gs_rasterize_forward_begin / _end, reference: RasterizeGaussiansCUDA, rasterize_points.cu:35-95) and
// the semantic render's recolor (gs_render_recolor) — in C++: the structs filled from at::Tensor
// accessors, the geometry / binning / image buffers allocated by at::empty from the allocator callback
// (no Python callback), argument checks as _C.py's.  The library is the instance dge_amd._native loaded:
// its entry points arrive as addresses (bind), so its state (binning capacity history, read-back slots,
// stage profiler) is shared with the ctypes path.  Errors come back as the C ABI's status code, which
// dge_amd._C turns into its usual NativeError.
#include <torch/extension.h>

#include <c10/core/DeviceGuard.h>

#include <cstdint>
#include <memory>
#include <unordered_map>

#include "gs_raster.h"

namespace {

struct Api {
    decltype(&gs_rasterize_forward_begin) begin = nullptr;
    decltype(&gs_rasterize_forward_end) end = nullptr;
    decltype(&gs_rasterize_forward_release) release = nullptr;
    decltype(&gs_render_recolor) recolor = nullptr;
    decltype(&gs_image_buffer_size) image_buffer_size = nullptr;
} api;

template <class F>
void take(const py::dict& fns, const char* name, F& dst) {
    if (!fns.contains(name)) throw std::runtime_error(std::string("gs_torch.bind: missing ") + name);
    dst = reinterpret_cast<F>(static_cast<uintptr_t>(fns[name].cast<uint64_t>()));
}

void bind(const py::dict& fns) {
    take(fns, "gs_rasterize_forward_begin", api.begin);
    take(fns, "gs_rasterize_forward_end", api.end);
    take(fns, "gs_rasterize_forward_release", api.release);
    take(fns, "gs_render_recolor", api.recolor);
    take(fns, "gs_image_buffer_size", api.image_buffer_size);
}

inline const void* ptr(const at::Tensor& t) { return t.defined() && t.numel() ? t.data_ptr() : nullptr; }
inline const float* fptr(const at::Tensor& t) { return static_cast<const float*>(ptr(t)); }

// _C._f32: a contiguous float32 tensor (or an absent one as is)
at::Tensor f32(const at::Tensor& t, const char* name) {
    if (!t.defined() || t.numel() == 0) return t;
    TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32 (got ", t.scalar_type(), ")");
    return t.contiguous();
}

// _C._features: fp32, or fp16 read as such (gs_params.sh_half)
at::Tensor features(const at::Tensor& t, const char* name) {
    if (!t.defined() || t.numel() == 0 || t.scalar_type() != at::kHalf) return f32(t, name);
    return t.contiguous();
}

// _C._f32_cached: the cameras' transposed 4x4 matrices are not contiguous; their contiguous copy is reused
// while the source tensor is alive and unmodified (same object, same version counter)
struct CacheEnt {
    c10::weak_intrusive_ptr<c10::TensorImpl> src;
    int64_t version;
    at::Tensor copy;
};
std::unordered_map<const c10::TensorImpl*, CacheEnt> g_contig;

at::Tensor f32_cached(const at::Tensor& t, const char* name) {
    if (!t.defined() || t.numel() == 0 || t.is_contiguous()) return f32(t, name);
    const c10::TensorImpl* key = t.unsafeGetTensorImpl();
    auto it = g_contig.find(key);
    if (it != g_contig.end()) {
        auto alive = it->second.src.lock();
        if (alive.get() == key && it->second.version == t._version()) return it->second.copy;
    }
    if (g_contig.size() > 256) {  // (drop the entries whose tensors are gone)
        for (auto i = g_contig.begin(); i != g_contig.end();) i = i->second.src.expired() ? g_contig.erase(i) : ++i;
    }
    at::Tensor c = f32(t, name);
    g_contig.erase(key);
    g_contig.emplace(key, CacheEnt{c10::weak_intrusive_ptr<c10::TensorImpl>(t.getIntrusivePtr()), t._version(), c});
    return c;
}

gs_settings settings(const at::Tensor& bg, const at::Tensor& view, const at::Tensor& proj, const at::Tensor& campos,
                     double tanfovx, double tanfovy, int64_t H, int64_t W, int64_t deg, double scale_modifier,
                     bool prefiltered, bool debug, std::vector<at::Tensor>& keep) {
    keep.push_back(f32(bg, "bg"));
    keep.push_back(f32_cached(view, "viewmatrix"));
    keep.push_back(f32_cached(proj, "projmatrix"));
    keep.push_back(f32_cached(campos, "campos"));
    gs_settings s{};
    s.image_height = (int)H;
    s.image_width = (int)W;
    s.tanfovx = (float)tanfovx;
    s.tanfovy = (float)tanfovy;
    s.bg = fptr(keep[keep.size() - 4]);
    s.scale_modifier = (float)scale_modifier;
    s.viewmatrix = fptr(keep[keep.size() - 3]);
    s.projmatrix = fptr(keep[keep.size() - 2]);
    s.sh_degree = (int)deg;
    s.campos = fptr(keep[keep.size() - 1]);
    s.prefiltered = prefiltered ? 1 : 0;
    s.debug = debug ? 1 : 0;
    return s;
}

// gs_alloc_fn: the torch caching allocator on the device's current stream (as _C._alloc_cb)
struct Alloc {
    int device = 0;
    at::Tensor buf[3];
};

void* alloc_cb(void* ctx, int which, size_t nbytes) {
    Alloc* a = static_cast<Alloc*>(ctx);
    if (which < 0 || which > 2) return nullptr;
    at::Tensor t = at::empty({(int64_t)nbytes}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, a->device));
    a->buf[which] = t;
    return nbytes ? t.data_ptr() : nullptr;
}

at::Tensor empty_u8(int device) {
    return at::empty({0}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, device));
}

// A raw-parameter forward between _begin and _end (_C.Prepared): the native handle, the allocator holding
// its buffers, its radii and every input it reads.  A handle never ended is released with the object.
struct Prepared {
    gs_forward_state* handle = nullptr;
    Alloc alloc;
    at::Tensor radii;
    std::vector<at::Tensor> keep;
    int64_t H = 0, W = 0, P = 0;
    int rc = 0;
    ~Prepared() {
        if (handle && api.release) api.release(handle);
    }
};

std::shared_ptr<Prepared> fused_begin(const at::Tensor& bg, const at::Tensor& xyz_in, const at::Tensor& f_dc_in,
                                      const at::Tensor& f_rest_in, const at::Tensor& colors_in, const at::Tensor& op_in,
                                      const at::Tensor& sc_in, const at::Tensor& rot_in, double scale_modifier,
                                      const at::Tensor& view, const at::Tensor& proj, double tanfovx, double tanfovy,
                                      int64_t H, int64_t W, int64_t deg, const at::Tensor& campos, bool prefiltered,
                                      bool debug, const c10::optional<at::Tensor>& index_in,
                                      const c10::optional<at::Tensor>& visible, bool forward_only,
                                      const c10::optional<at::Tensor>& aux_in, int64_t stream) {
    TORCH_CHECK(xyz_in.is_cuda(), "dge_amd: tensors must live on the GPU");
    const int dev = xyz_in.get_device();
    c10::DeviceGuard guard(xyz_in.device());
    auto p = std::make_shared<Prepared>();
    p->alloc.device = dev;
    at::Tensor index;
    if (index_in && index_in->defined()) {
        TORCH_CHECK(index_in->scalar_type() == at::kInt && index_in->dim() == 1,
                    "index must be a 1-D int32 tensor of parameter rows");
        index = index_in->contiguous();
    }
    const int64_t P = index.defined() ? index.numel() : xyz_in.size(0);
    at::Tensor xyz = f32(xyz_in, "xyz");
    at::Tensor f_dc = features(f_dc_in, "features_dc"), f_rest = features(f_rest_in, "features_rest");
    at::Tensor colors = f32(colors_in, "colors");
    at::Tensor op = f32(op_in, "opacity"), sc = f32(sc_in, "scaling"), rot = f32(rot_in, "rotation");
    p->radii = at::empty({P}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, dev));
    at::Tensor aux;
    if (aux_in && aux_in->defined()) {
        TORCH_CHECK((aux_in->scalar_type() == at::kBool || aux_in->scalar_type() == at::kByte) &&
                        aux_in->get_device() == dev && aux_in->dim() == 1 && aux_in->numel() == xyz.size(0),
                    "aux_mask must be a bool or uint8 tensor over the parameter rows, on the device");
        aux = aux_in->contiguous().view(at::kByte);
    }
    // gs_params of the raw-parameter path (_C._params)
    gs_params g{};
    g.P = (int)P;
    g.forward_only = forward_only ? 1 : 0;
    g.aux_mask = aux.defined() ? static_cast<const uint8_t*>(aux.data_ptr()) : nullptr;
    g.index = index.defined() ? static_cast<const int*>(ptr(index)) : nullptr;
    g.sh_half = f_dc.defined() && f_dc.scalar_type() == at::kHalf ? 1 : 0;
    const bool have_sh = f_dc.defined() && f_dc.numel() != 0;
    const int Mr = have_sh && f_rest.defined() && f_rest.numel() != 0 ? (int)f_rest.size(1) : 0;
    g.M = have_sh ? 1 + Mr : 0;
    g.means3D = fptr(xyz);
    g.sh_dc = have_sh ? fptr(f_dc) : nullptr;
    g.sh_rest = Mr ? fptr(f_rest) : nullptr;
    g.sh_dc_stride = 3;
    g.sh_rest_stride = 3 * Mr;
    g.colors_precomp = have_sh ? nullptr : fptr(colors);
    g.opacities = fptr(op);
    g.scales = fptr(sc);
    g.rotations = fptr(rot);
    g.cov3D_precomp = nullptr;
    g.activation = 1;
    if (visible && visible->defined()) {
        TORCH_CHECK(visible->scalar_type() == at::kBool && visible->numel() == P && visible->is_contiguous(),
                    "visible must be a contiguous bool tensor of P elements");
        g.visible_out = static_cast<uint8_t*>(visible->data_ptr());
    }
    std::vector<at::Tensor>& keep = p->keep;
    const gs_settings s = settings(bg, view, proj, campos, tanfovx, tanfovy, H, W, deg, scale_modifier, prefiltered,
                                   debug, keep);
    for (const at::Tensor* t : {&xyz, &f_dc, &f_rest, &colors, &op, &sc, &rot, &index, &aux})
        if (t->defined()) keep.push_back(*t);
    if (visible && visible->defined()) keep.push_back(*visible);
    const at::Tensor e = empty_u8(dev);
    for (auto& b : p->alloc.buf) b = e;
    p->H = H;
    p->W = W;
    p->P = P;
    gs_forward_state* h = nullptr;
    p->rc = api.begin(&s, &g, static_cast<int*>(p->radii.data_ptr()), alloc_cb, &p->alloc,
                      reinterpret_cast<gs_stream_t>(static_cast<uintptr_t>(stream)), &h);
    p->handle = p->rc ? nullptr : h;
    return p;
}

// -> (rc, num_rendered, color, depth, radii, geom, binning, img)
py::tuple fused_end(const std::shared_ptr<Prepared>& p, int64_t stream) {
    TORCH_CHECK(p->handle, "rasterize_gaussians_fused_end: the forward was not begun, or already ended");
    c10::DeviceGuard guard(p->radii.device());
    const auto opts = at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, p->alloc.device);
    at::Tensor color = at::empty({3, p->H, p->W}, opts), depth = at::empty({1, p->H, p->W}, opts);
    gs_forward_state* h = p->handle;
    p->handle = nullptr;  // (_end consumes the handle, also on error)
    int nr = 0;
    const int rc = api.end(h, static_cast<float*>(color.data_ptr()), static_cast<float*>(depth.data_ptr()), alloc_cb,
                           &p->alloc, reinterpret_cast<gs_stream_t>(static_cast<uintptr_t>(stream)), &nr);
    if (p->P == 0) p->radii.zero_();
    return py::make_tuple(rc, nr, color, depth, p->radii, p->alloc.buf[0], p->alloc.buf[1], p->alloc.buf[2]);
}

// -> (rc, color, depth)   (_C.render_recolor)
py::tuple render_recolor(const at::Tensor& bg, const at::Tensor& colors_in, const at::Tensor& view,
                         const at::Tensor& proj, const at::Tensor& campos, double tanfovx, double tanfovy, int64_t H,
                         int64_t W, int64_t deg, double scale_modifier, bool prefiltered, int64_t P,
                         int64_t num_rendered, const at::Tensor& geom, const at::Tensor& binning,
                         const at::Tensor& img, const c10::optional<at::Tensor>& src_aux, int64_t stream) {
    const int dev = colors_in.get_device();
    c10::DeviceGuard guard(colors_in.device());
    at::Tensor colors = f32(colors_in, "colors");
    TORCH_CHECK(colors.numel() >= 3 * P, "colors must hold P x 3 values");
    std::vector<at::Tensor> keep;
    const gs_settings s = settings(bg, view, proj, campos, tanfovx, tanfovy, H, W, deg, scale_modifier, prefiltered,
                                   false, keep);
    const auto opts = at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev);
    at::Tensor color = at::empty({3, H, W}, opts), depth = at::empty({1, H, W}, opts);
    at::Tensor img_out = at::empty({(int64_t)api.image_buffer_size((int)W, (int)H)},
                                   at::TensorOptions().dtype(at::kByte).device(at::kCUDA, dev));
    at::Tensor src;
    if (src_aux && src_aux->defined()) {
        src = src_aux->contiguous().view(at::kByte);
        TORCH_CHECK(src.numel() >= P, "src_aux_mask must cover the P Gaussians");
    }
    const int rc = api.recolor(&s, (int)P, (int)num_rendered, ptr(geom), ptr(binning), ptr(img), fptr(colors),
                               img_out.data_ptr(), static_cast<float*>(color.data_ptr()),
                               static_cast<float*>(depth.data_ptr()),
                               src.defined() ? static_cast<const uint8_t*>(src.data_ptr()) : nullptr,
                               reinterpret_cast<gs_stream_t>(static_cast<uintptr_t>(stream)));
    return py::make_tuple(rc, color, depth);
}

}  // namespace

PYBIND11_MODULE(_gs_torch, m) {
    m.doc() = "compiled torch binding of the per-view render() path of libgs_raster.so (include/gs_raster.h)";
    m.def("bind", &bind, "take the C ABI's entry points (name -> address) from the loaded library");
    py::class_<Prepared, std::shared_ptr<Prepared>>(m, "Prepared", py::dynamic_attr())
        .def_readonly("rc", &Prepared::rc)
        .def_readonly("radii", &Prepared::radii)
        .def_readonly("P", &Prepared::P)
        .def_property_readonly("open", [](const Prepared& p) { return p.handle != nullptr; });
    m.def("fused_begin", &fused_begin);
    m.def("fused_end", &fused_end);
    m.def("render_recolor", &render_recolor);
}
