// bbm_amd/csrc/parse.hip -- model strings -> registry entries (host code only).
//
// The reference's runtime entry point for "a BSDF named by a string" is bsdf_ptr fromString
// (include/bbm/bsdf_string_convert.h:52-85: keyword lookup over every exported model plus aggregatebsdf),
// used by checkBsdf (bin/checkBsdf.cpp:435-479), the Mitsuba plugin and the .fit files.  bbm_hip_parse_model
// restates it for the C-ABI: `Name(attr = value, ...)` (attributes by name in any order, or positionally in
// declaration order; missing ones keep their defaults; a scalar broadcasts over an RGB / Vec2d attribute) and
// `Aggregate(child, child, ...)`, nested to any depth.  A single model or an Aggregate(Lambertian, X) with a fused
// kernel is one registry entry; any other aggregate is a composed node whose children are entries or composed
// nodes again, for the composed path (bbm_hip_aggregate_*): bbm_hip_parse_model returns one level, and
// bbm_hip_parse_model_tree the whole tree in preorder.
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

// A parsed model: a registry entry (single model or fused aggregate) with its parameters, or a composed
// aggregate (kids.size() >= 2) whose children are nodes again -- aggregatemodel_base takes any bsdfmodel child
// (aggregatemodel.h:22), including another aggregate, and keeps it as one child: its eval / pdf / sample /
// reflectance stay the inner aggregate's own (no flattening, which would change the fold order and the sampling).
struct Node
{
  Child leaf;
  std::vector<Node> kids;
  bool composed() const { return !kids.empty(); }
};

bool parse_any(Parser& p, Node& node, int& code)
{
  const std::string name = p.ident();
  if (name.empty()) { code = BBM_HIP_ERR_INVALID_ARG; p.err = "malformed BSDF string"; return false; }
  if (name != "Aggregate") return parse_single(p, name, node.leaf, code);
  if (!p.eat('(')) { code = BBM_HIP_ERR_INVALID_ARG; p.err = "Aggregate: expected '('"; return false; }
  std::vector<Node> sub;
  do
  {
    sub.emplace_back();
    if (!parse_any(p, sub.back(), code)) return false;
  } while (p.eat(','));
  if (!p.eat(')')) { code = BBM_HIP_ERR_INVALID_ARG; p.err = "Aggregate: expected ')'"; return false; }
  if (sub.size() < 2) { code = BBM_HIP_ERR_INVALID_ARG; p.err = "Aggregate: needs at least two models"; return false; }
  // a fused kernel for exactly this composition of registry entries (the fits' Aggregate(Lambertian, X))?
  bool flat = true;
  std::string key = "Aggregate<";
  for (size_t k = 0; k < sub.size(); ++k)
  {
    flat = flat && !sub[k].composed();
    key += (k ? "," : "") + sub[k].leaf.name;
  }
  key += ">";
  const int fid = flat ? bbm_hip_model_id(key.c_str()) : -1;
  if (fid >= 0)
  {
    node.leaf.name = key;
    for (const auto& k : sub) node.leaf.params.insert(node.leaf.params.end(), k.leaf.params.begin(), k.leaf.params.end());
  }
  else node.kids = std::move(sub);
  return true;
}

// registry id of a parsed leaf: every "Aggregate(...)" of a string is the runtime aggregatebsdf
// (bsdf_string_convert.h:59), so a fused aggregate's id carries BBM_HIP_RUNTIME_AGGREGATE
int string_id(const std::string& name)
{
  const int id = bbm_hip_model_id(name.c_str());
  return (id >= 0 && name.rfind("Aggregate<", 0) == 0) ? (id | BBM_HIP_RUNTIME_AGGREGATE) : id;
}

// preorder flattening for bbm_hip_parse_model_tree
void preorder(const Node& n, std::vector<const Node*>& out)
{
  out.push_back(&n);
  for (const auto& k : n.kids) preorder(k, out);
}

bool parse_root(const std::string& s, Node& root, int& rc)
{
  Parser p(s);
  int code = BBM_HIP_OK;
  if (!parse_any(p, root, code)) { rc = fail(code, p.err.empty() ? "malformed BSDF string: " + s : p.err); return false; }
  p.ws();
  if (p.i != s.size()) { rc = fail(BBM_HIP_ERR_INVALID_ARG, "malformed BSDF string (trailing text): " + s); return false; }
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
  Node root;
  int rc = BBM_HIP_OK;
  if (!parse_root(s, root, rc)) return rc;
  std::vector<const Child*> kids;
  if (!root.composed()) kids.push_back(&root.leaf);
  for (const auto& k : root.kids)
  {
    if (k.composed())
      return fail(BBM_HIP_ERR_UNSUPPORTED, "a composed aggregate nested in another: use bbm_hip_parse_model_tree (" + s + ")");
    kids.push_back(&k.leaf);
  }
  if (int(kids.size()) > max_children)
    return fail(BBM_HIP_ERR_INVALID_ARG, "too many children for the output arrays (" + std::to_string(kids.size()) + ")");
  int total = 0;
  for (const Child* k : kids) total += int(k->params.size());
  if (total > params_capacity) return fail(BBM_HIP_ERR_INVALID_ARG, "params capacity too small (" + std::to_string(total) + ")");
  int off = 0;
  for (size_t c = 0; c < kids.size(); ++c)
  {
    if (model_ids) model_ids[c] = string_id(kids[c]->name);
    if (nparams) nparams[c] = int(kids[c]->params.size());
    for (float v : kids[c]->params) if (params) params[off++] = v;
  }
  return int(kids.size());
}

int bbm_hip_parse_model_tree(const char* str, int* model_ids, int* nchildren, float* params, int* nparams,
                             int max_nodes, int params_capacity)
{
  if (!str) return fail(BBM_HIP_ERR_INVALID_ARG, "string is NULL");
  const std::string s(str);
  Node root;
  int rc = BBM_HIP_OK;
  if (!parse_root(s, root, rc)) return rc;
  std::vector<const Node*> nodes;
  preorder(root, nodes);
  if (int(nodes.size()) > max_nodes)
    return fail(BBM_HIP_ERR_INVALID_ARG, "too many nodes for the output arrays (" + std::to_string(nodes.size()) + ")");
  int total = 0;
  for (const Node* n : nodes) total += int(n->leaf.params.size());
  if (total > params_capacity) return fail(BBM_HIP_ERR_INVALID_ARG, "params capacity too small (" + std::to_string(total) + ")");
  int off = 0;
  for (size_t k = 0; k < nodes.size(); ++k)
  {
    const Node& n = *nodes[k];
    if (model_ids) model_ids[k] = n.composed() ? BBM_HIP_AGGREGATE_BSDF : string_id(n.leaf.name);
    if (nchildren) nchildren[k] = int(n.kids.size());
    if (nparams) nparams[k] = int(n.leaf.params.size());
    for (float v : n.leaf.params) if (params) params[off++] = v;
  }
  return int(nodes.size());
}

}  // extern "C"
