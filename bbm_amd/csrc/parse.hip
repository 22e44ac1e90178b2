// bbm_amd/csrc/parse.hip -- model strings -> registry entries (host code only).
//
// The reference's runtime entry point for "a BSDF named by a string" is bsdf_ptr fromString
// (include/bbm/bsdf_string_convert.h:52-85: keyword lookup over every exported model plus aggregatebsdf),
// used by checkBsdf (bin/checkBsdf.cpp:435-479), the Mitsuba plugin and the .fit files.  bbm_hip_parse_model
// restates it for the C-ABI: `Name(attr = value, ...)` (attributes by name in any order, or positionally in
// declaration order; missing ones keep their defaults; a scalar broadcasts over an RGB / Vec2d attribute) and
// `Aggregate(child, child, ...)`.  A single model or an Aggregate(Lambertian, X) with a fused kernel yields one
// registry entry; any other aggregate yields its children, for the composed path (bbm_hip_aggregate_*).
// Errors follow the reference's std::invalid_argument cases (unknown name, malformed string, unknown
// attribute, wrong value count) plus std::out_of_range (a value beyond the float range).
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bbm_hip.h"

namespace bbmhip {
int fail(int code, const std::string& msg);

namespace {

// attribute layouts in declaration order (bbm::reflection::attributes, the order toString prints and
// parameter_values packs), "name:count" with count = product of the attribute's shape
struct Layout { const char* model; const char* attrs; };
const Layout kLayouts[] = {
  {"Lambertian", "albedo:3"},
  {"OrenNayar", "albedo:3,roughness:1"},
  {"CookTorrance", "albedo:3,roughness:1,eta:1"},
  {"CookTorranceHeitz", "albedo:3,roughness:2,eta:1"},
  {"CookTorranceWalter", "albedo:3,roughness:1,eta:1"},
  {"GGX", "albedo:3,roughness:1,eta:1"},
  {"GGXHeitz", "albedo:3,roughness:2,eta:1"},
  {"PhongWalter", "albedo:3,sharpness:1,eta:1"},
  {"Ribardiere", "albedo:3,roughness:1,gamma:1,eta:1"},
  {"RibardiereAnisotropic", "albedo:3,roughness:2,gamma:1,eta:1"},
  {"Bagher", "albedo:3,K:3,Lambda:3,c:3,theta0:3,k:3,alpha:3,p:3,eta:6"},
  {"LowCookTorrance", "albedo:3,roughness:1,eta:1"},
  {"LowMicrofacet", "A:3,B:1,C:1,eta:1"},
  {"LowMicrofacetFit", "A:3,B:1,C:1,eta:1"},
  {"NganCookTorrance", "albedo:3,roughness:1,eta:1"},
  {"Ward", "albedo:3,roughness:2"},
  {"WardDuer", "albedo:3,roughness:2"},
  {"WardDuerGeislerMoroder", "albedo:3,roughness:2"},
  {"NganWard", "albedo:3,roughness:1"},
  {"NganWardDuer", "albedo:3,roughness:1"},
  {"Phong", "albedo:3,sharpness:1"},
  {"NganBlinnPhong", "albedo:3,sharpness:1"},
  {"Lafortune", "albedo:3,Cxy:2,Cz:1,sharpness:1"},
  {"NganLafortune", "albedo:3,Cxy:1,Cz:1,sharpness:1"},
  {"AshikhminShirley", "fresnelReflectance:3,sharpness:2"},
  {"AshikhminShirleyFull", "diffuseReflectance:3,fresnelReflectance:3,sharpness:2"},
  {"LowAshikhminShirley", "albedo:3,fresnelReflectance:1,sharpness:1"},
  {"NganAshikhminShirley", "albedo:3,fresnelReflectance:1,sharpness:1"},
  {"LowSmooth", "A:3,B:1,C:1,eta:1"},
  {"EPD", "beta:1,p:1,eta:2"},
  {"He", "roughness:1,autocorrelation:1,eta:6"},
  {"HeWestin", "roughness:1,autocorrelation:1,eta:6"},
  {"HeHolzschuch", "roughness:1,autocorrelation:1,eta:6"},
  {"NganHe", "albedo:3,roughness:1,autocorrelation:1,eta:1"},
};

const char* layout_of(const std::string& model)
{
  for (const auto& l : kLayouts)
    if (model == l.model) return l.attrs;
  return nullptr;
}

struct Attr { std::string name; int count; };

std::vector<Attr> split_layout(const char* s)
{
  std::vector<Attr> out;
  std::string cur(s);
  size_t pos = 0;
  while (pos < cur.size())
  {
    const size_t comma = cur.find(',', pos);
    const std::string item = cur.substr(pos, comma == std::string::npos ? std::string::npos : comma - pos);
    const size_t colon = item.find(':');
    out.push_back({item.substr(0, colon), std::atoi(item.c_str() + colon + 1)});
    if (comma == std::string::npos) break;
    pos = comma + 1;
  }
  return out;
}

struct Parser
{
  const std::string& s;
  size_t i = 0;
  std::string err;

  explicit Parser(const std::string& str) : s(str) {}
  void ws() { while (i < s.size() && std::isspace(static_cast<unsigned char>(s[i]))) ++i; }
  bool eat(char c) { ws(); if (i < s.size() && s[i] == c) { ++i; return true; } return false; }
  bool peek(char c) { ws(); return i < s.size() && s[i] == c; }
  std::string ident()
  {
    ws();
    const size_t b = i;
    if (i < s.size() && (std::isalpha(static_cast<unsigned char>(s[i])) || s[i] == '_'))
      while (i < s.size() && (std::isalnum(static_cast<unsigned char>(s[i])) || s[i] == '_')) ++i;
    return s.substr(b, i - b);
  }
  // a number or a (nested) bracketed list, flattened
  bool value(std::vector<double>& out)
  {
    if (eat('['))
    {
      if (eat(']')) return true;
      do { if (!value(out)) return false; } while (eat(','));
      if (!eat(']')) { err = "expected ']'"; return false; }
      return true;
    }
    ws();
    const char* b = s.c_str() + i;
    char* e = nullptr;
    const double v = std::strtod(b, &e);
    if (e == b) { err = "expected a number at: " + s.substr(i, 20); return false; }
    i += size_t(e - b);
    out.push_back(v);
    return true;
  }
};

struct Child { std::string name; std::vector<float> params; };

// Name(attr = v, ...) with the defaults of the registry entry filled in first
bool parse_single(Parser& p, const std::string& name, Child& out, int& code)
{
  const char* lay = layout_of(name);
  const int id = lay ? bbm_hip_model_id(name.c_str()) : -1;
  if (!lay || id < 0) { code = BBM_HIP_ERR_INVALID_MODEL; p.err = "unknown BSDF model: " + name; return false; }
  const std::vector<Attr> attrs = split_layout(lay);
  const int np = bbm_hip_model_nparams(id);
  out.name = name;
  out.params.assign(size_t(np), 0.0f);
  bbm_hip_model_params(id, 0, out.params.data(), np);
  if (!p.eat('(')) return true;          // bare name: defaults
  size_t positional = 0;
  if (p.eat(')')) return true;
  do
  {
    const size_t save = p.i;
    std::string key = p.ident();
    size_t which = attrs.size();
    if (!key.empty() && p.eat('='))
    {
      for (size_t a = 0; a < attrs.size(); ++a) if (attrs[a].name == key) which = a;
      if (which == attrs.size()) { code = BBM_HIP_ERR_INVALID_ARG; p.err = name + ": unknown attribute '" + key + "'"; return false; }
    }
    else
    {
      p.i = save;
      which = positional;
      if (which >= attrs.size()) { code = BBM_HIP_ERR_INVALID_ARG; p.err = name + ": too many attributes"; return false; }
    }
    ++positional;
    std::vector<double> v;
    if (!p.value(v)) { code = BBM_HIP_ERR_INVALID_ARG; return false; }
    const int n = attrs[which].count;
    if (int(v.size()) != n && v.size() != 1)
    {
      code = BBM_HIP_ERR_INVALID_ARG;
      p.err = name + "." + attrs[which].name + ": expected " + std::to_string(n) + " values, got " + std::to_string(v.size());
      return false;
    }
    int off = 0;
    for (size_t a = 0; a < which; ++a) off += attrs[a].count;
    for (int k = 0; k < n; ++k)
    {
      const double d = v[v.size() == 1 ? 0 : size_t(k)];
      const float f = float(d);
      if (std::isfinite(d) && !std::isfinite(f))
      {
        code = BBM_HIP_ERR_INVALID_ARG;
        p.err = name + "." + attrs[which].name + ": value out of the float range";
        return false;
      }
      out.params[size_t(off + k)] = f;
    }
  } while (p.eat(','));
  if (!p.eat(')')) { code = BBM_HIP_ERR_INVALID_ARG; p.err = "malformed BSDF string: expected ')' in " + name; return false; }
  return true;
}

bool parse_any(Parser& p, std::vector<Child>& kids, int& code)
{
  const std::string name = p.ident();
  if (name.empty()) { code = BBM_HIP_ERR_INVALID_ARG; p.err = "malformed BSDF string"; return false; }
  if (name != "Aggregate")
  {
    kids.emplace_back();
    return parse_single(p, name, kids.back(), code);
  }
  if (!p.eat('(')) { code = BBM_HIP_ERR_INVALID_ARG; p.err = "Aggregate: expected '('"; return false; }
  std::vector<Child> sub;
  do
  {
    if (!parse_any(p, sub, code)) return false;
  } while (p.eat(','));
  if (!p.eat(')')) { code = BBM_HIP_ERR_INVALID_ARG; p.err = "Aggregate: expected ')'"; return false; }
  if (sub.size() < 2) { code = BBM_HIP_ERR_INVALID_ARG; p.err = "Aggregate: needs at least two models"; return false; }
  // a fused kernel for exactly this composition (the fits' Aggregate(Lambertian, X))?
  std::string key = "Aggregate<";
  for (size_t k = 0; k < sub.size(); ++k) key += (k ? "," : "") + sub[k].name;
  key += ">";
  const int fid = bbm_hip_model_id(key.c_str());
  if (fid >= 0)
  {
    Child c;
    c.name = key;
    for (const auto& k : sub) c.params.insert(c.params.end(), k.params.begin(), k.params.end());
    kids.push_back(c);
  }
  else
  {
    for (const auto& k : sub)
      if (k.name.rfind("Aggregate<", 0) == 0)
      {
        code = BBM_HIP_ERR_UNSUPPORTED;
        p.err = "nested aggregate without a fused kernel: " + k.name;
        return false;
      }
    kids.insert(kids.end(), sub.begin(), sub.end());
  }
  return true;
}

}  // namespace
}  // namespace bbmhip

using namespace bbmhip;

extern "C" {

const char* bbm_hip_model_layout(int model_id)
{
  const char* name = bbm_hip_model_name(model_id);
  if (!name) { fail(BBM_HIP_ERR_INVALID_MODEL, "unknown model id " + std::to_string(model_id)); return nullptr; }
  return layout_of(name);
}

int bbm_hip_parse_model(const char* str, int* model_ids, float* params, int* nparams, int max_children,
                        int params_capacity)
{
  if (!str) return fail(BBM_HIP_ERR_INVALID_ARG, "string is NULL");
  const std::string s(str);
  Parser p(s);
  std::vector<Child> kids;
  int code = BBM_HIP_OK;
  if (!parse_any(p, kids, code)) return fail(code, p.err.empty() ? "malformed BSDF string: " + s : p.err);
  p.ws();
  if (p.i != s.size()) return fail(BBM_HIP_ERR_INVALID_ARG, "malformed BSDF string (trailing text): " + s);
  if (int(kids.size()) > max_children)
    return fail(BBM_HIP_ERR_INVALID_ARG, "too many children for the output arrays (" + std::to_string(kids.size()) + ")");
  int total = 0;
  for (const auto& k : kids) total += int(k.params.size());
  if (total > params_capacity) return fail(BBM_HIP_ERR_INVALID_ARG, "params capacity too small (" + std::to_string(total) + ")");
  int off = 0;
  for (size_t c = 0; c < kids.size(); ++c)
  {
    if (model_ids) model_ids[c] = bbm_hip_model_id(kids[c].name.c_str());
    if (nparams) nparams[c] = int(kids[c].params.size());
    for (float v : kids[c].params) if (params) params[off++] = v;
  }
  return int(kids.size());
}

}  // extern "C"
