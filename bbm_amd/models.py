"""Host-side mirror of BBM's model registry and attribute reflection.

In the reference every model is a template whose attributes are reflected at compile time
(BBM_ATTRIBUTES, include/util/reflection.h) and whose name is registered by
BBM_EXPORT_BSDFMODEL (e.g. include/bsdfmodel/cooktorrance.h:42).  The Python bindings expose a
constructor per model name taking the attributes as keyword arguments
(include/python/py_bsdf.h:67-80) and `str()` prints bbm::toString
(e.g. `CookTorrance(albedo = [0.5, 0.5, 0.5], roughness = 0.1, eta = 1.3)`).

Here the attribute *layout* (names and shapes, in declaration order) lives in this table; the
default values and bounds come from libbbm_hip itself (bbm_hip_model_params) so the library is
the single source of truth for what the kernels expect.  Both are pinned against the reference itself
(oracle/_ref: tests/test_abi.py::test_registry_matches_reference, ::test_python_mirror_layout_covers_every_reference_model,
::test_param_attrs_match_reference).
"""

# attribute layout per model: list of (name, shape); shape () = scalar, (3,) = RGB/Spectrum,
# (2,) = anisotropic Vec2d, (2, 3) = complex Spectrum ([real RGB], [imag RGB]).
# Reference: the BBM_ATTRIBUTES(...) of each include/bsdfmodel/*.h (+ scaledmodel albedo first,
# bsdfmodel/scaledmodel.h:71-74; microfacet NDF attributes then eta, microfacet.h:197-200).
RGB, V2, S, CRGB = (3,), (2,), (), (2, 3)

ATTRIBUTES = {
    "Lambertian": [("albedo", RGB)],                                                      # lambertian.h
    "OrenNayar": [("albedo", RGB), ("roughness", S)],                                     # orennayar.h
    "CookTorrance": [("albedo", RGB), ("roughness", S), ("eta", S)],                      # cooktorrance.h:28-34
    "CookTorranceHeitz": [("albedo", RGB), ("roughness", V2), ("eta", S)],                # cooktorranceheitz.h:33-39
    "CookTorranceWalter": [("albedo", RGB), ("roughness", S), ("eta", S)],                # cooktorrancewalter.h:32-38
    "GGX": [("albedo", RGB), ("roughness", S), ("eta", S)],                               # ggx.h:27-33
    "GGXHeitz": [("albedo", RGB), ("roughness", V2), ("eta", S)],                         # ggxheitz.h:28-34
    "PhongWalter": [("albedo", RGB), ("sharpness", S), ("eta", S)],                       # phongwalter.h:27-33
    "Ribardiere": [("albedo", RGB), ("roughness", S), ("gamma", S), ("eta", S)],          # ribardiere.h:28-34
    "RibardiereAnisotropic": [("albedo", RGB), ("roughness", V2), ("gamma", S), ("eta", S)],  # ribardiere.h:46-52
    "Bagher": [("albedo", RGB), ("K", RGB), ("Lambda", RGB), ("c", RGB), ("theta0", RGB), ("k", RGB),
               ("alpha", RGB), ("p", RGB), ("eta", CRGB)],                                 # bagher.h:38-68, ndf/sgd.h
    "LowCookTorrance": [("albedo", RGB), ("roughness", S), ("eta", S)],                   # low.h:32-33
    "LowMicrofacet": [("A", RGB), ("B", S), ("C", S), ("eta", S)],                         # lowmicrofacet.h:38-95
    "LowMicrofacetFit": [("A", RGB), ("B", S), ("C", S), ("eta", S)],                      # low.h:40-41
    "NganCookTorrance": [("albedo", RGB), ("roughness", S), ("eta", S)],                  # ngan.h:141-147
    "Ward": [("albedo", RGB), ("roughness", V2)],                                          # ward.h:26-168
    "WardDuer": [("albedo", RGB), ("roughness", V2)],                                      # wardduer.h:29-81
    "WardDuerGeislerMoroder": [("albedo", RGB), ("roughness", V2)],                        # wardduergeislermoroder.h:29-81
    "NganWard": [("albedo", RGB), ("roughness", S)],                                       # ngan.h:30-31
    "NganWardDuer": [("albedo", RGB), ("roughness", S)],                                   # ngan.h:37-38
    "Phong": [("albedo", RGB), ("sharpness", S)],                                          # phong.h:25-163
    "NganBlinnPhong": [("albedo", RGB), ("sharpness", S)],                                 # ngan.h:43-44
    "Lafortune": [("albedo", RGB), ("Cxy", V2), ("Cz", S), ("sharpness", S)],              # lafortune.h:28-172
    "NganLafortune": [("albedo", RGB), ("Cxy", S), ("Cz", S), ("sharpness", S)],           # ngan.h:54-129
    "AshikhminShirley": [("fresnelReflectance", RGB), ("sharpness", V2)],                  # ashikhminshirley.h:29-221
    "AshikhminShirleyFull": [("diffuseReflectance", RGB), ("fresnelReflectance", RGB), ("sharpness", V2)],  # ashikhminshirleyfull.h
    "LowAshikhminShirley": [("albedo", RGB), ("fresnelReflectance", S), ("sharpness", S)],  # low.h:24-25
    "NganAshikhminShirley": [("albedo", RGB), ("fresnelReflectance", S), ("sharpness", S)],  # ngan.h:157-158
    "LowSmooth": [("A", RGB), ("B", S), ("C", S), ("eta", S)],                             # lowsmooth.h:17-194
    "EPD": [("beta", S), ("p", S), ("eta", V2)],            # holzschuchpacanowski.h:34-42, ndf/epd.h:180-182; eta = (n, k)
    "He": [("roughness", S), ("autocorrelation", S), ("eta", CRGB)],                        # he.h:473-477, :489-490
    "HeWestin": [("roughness", S), ("autocorrelation", S), ("eta", CRGB)],                  # he.h:492-493
    "HeHolzschuch": [("roughness", S), ("autocorrelation", S), ("eta", CRGB)],              # he.h:495-496
    "NganHe": [("albedo", RGB), ("roughness", S), ("autocorrelation", S), ("eta", S)],      # ngan.h:166-167
}


# Aggregate(Lambertian, X) registry keys -> children (aggregatemodel.h:22-233; the published fits'
# form, fits/*.fit).  Parameters are the children's vectors concatenated in order.
AGGREGATES = {f"Aggregate<Lambertian,{x}>": ("Lambertian", x) for x in (
    "Bagher", "CookTorrance", "GGX", "LowCookTorrance", "LowAshikhminShirley", "LowMicrofacetFit", "LowSmooth",
    "NganAshikhminShirley", "NganBlinnPhong", "NganCookTorrance", "NganLafortune", "NganWard", "NganWardDuer",
    "NganHe")}


def aggregate_key(children):
    return "Aggregate<" + ",".join(children) + ">"


def aggregate_children(name):
    """Children of an aggregate key: the fused entries' (AGGREGATES) or, for any other `Aggregate<A,B,...>` of
    single models (the composed path), the names in the key."""
    if name in AGGREGATES:
        return AGGREGATES[name]
    if name.startswith("Aggregate<") and name.endswith(">"):
        kids = tuple(name[len("Aggregate<"):-1].split(","))
        if len(kids) >= 2 and all(k in ATTRIBUTES for k in kids):
            return kids
    return None


def attr_size(shape):
    n = 1
    for d in shape:
        n *= d
    return n


def nparams(name):
    kids = aggregate_children(name)
    if kids is not None:
        return sum(nparams(c) for c in kids)
    return sum(attr_size(s) for _, s in ATTRIBUTES[name])


def fmt_value(v):
    """C++ ostream default formatting (precision 6, %g-like) used by bbm::toString."""
    return "%g" % float(v)


def fmt_attr(values, shape):
    if shape == ():
        return fmt_value(values[0])
    if len(shape) == 1:
        return "[" + ", ".join(fmt_value(v) for v in values) + "]"
    rows = [values[i * shape[1]:(i + 1) * shape[1]] for i in range(shape[0])]
    return "[" + ", ".join("[" + ", ".join(fmt_value(v) for v in r) + "]" for r in rows) + "]"


def to_string(name, params):
    """bbm::toString(model): `Name(attr = value, ...)` in attribute declaration order;
    aggregates print `Aggregate(child, child)` (aggregatemodel.h:168-179)."""
    kids = aggregate_children(name)
    if kids is not None:
        parts, k = [], 0
        for c in kids:
            n = nparams(c)
            parts.append(to_string(c, params[k:k + n]))
            k += n
        return "Aggregate(" + ", ".join(parts) + ")"
    parts, k = [], 0
    for attr, shape in ATTRIBUTES[name]:
        n = attr_size(shape)
        parts.append(f"{attr} = {fmt_attr(params[k:k + n], shape)}")
        k += n
    return f"{name}(" + ", ".join(parts) + ")"
