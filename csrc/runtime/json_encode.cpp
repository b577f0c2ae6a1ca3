// serde_json-compatible compact JSON text of a plain Python value tree (dict / list / tuple / str / int /
// float / bool / None), for the server's response bodies (utils/json.py dumps).
//
// The reference serialises with serde_json (compact, insertion-ordered maps) and formats f64 with ryu
// (/root/reference/src/score/completions/client.rs:1580-1603 for the text, Cargo.toml's serde_json +
// rust_decimal serde-float).  Python's own C encoder differs in float text (repr: 1e-05, ryu: 1e-5) and is
// slow on the score responses (~47 KB of logprob objects: 1.8 ms per response, most of it float repr and
// small ints); this walks the tree once with the CPython API and writes:
//   * floats: the shortest round-trip digits (std::to_chars — libstdc++ implements it with Ryu) laid out by
//     ryu's rules (decimal when the exponent allows, else d.ddde±x without '+'), "0.0" / "-0.0", non-finite
//     -> null (serde_json's behaviour) — the same text as utils/json.py ryu_f64;
//   * strings: serde_json escaping == json.dumps(ensure_ascii=False): \" \\ \b \f \n \r \t, other C0
//     controls as \u00xx (lowercase hex), everything else raw UTF-8;
//   * ints: decimal (arbitrary size through PyObject_Str on overflow); bool before int.
// Wire objects (schema/base.py) are written straight from their __dict__ by their field plan — declaration
// order, wire key (alias), None omitted unless kept — without building the to_obj() dict tree first (~800
// logprob objects per scored response).  ``plan_of(cls)`` gives the plan as ((name, key, keep_none), ...) or
// None for classes whose to_obj() is their own (overrides, flattened fields): those, and instances with
// extra fields, are written from to_obj().  Anything else raises TypeError and the caller takes the exact
// Python encoder.
#include <Python.h>
#include <pybind11/pybind11.h>

#include <charconv>
#include <cmath>
#include <cstring>
#include <string>

namespace py = pybind11;

namespace lwc {
namespace {

struct TypeErr {};

void put_f64(std::string& out, double x) {
  if (!std::isfinite(x)) {
    out += "null";
    return;
  }
  if (x == 0.0) {
    out += std::signbit(x) ? "-0.0" : "0.0";
    return;
  }
  char buf[64];
  // shortest round-trip digits in scientific form: [-]D[.DDDD]e[+-]XX
  auto r = std::to_chars(buf, buf + sizeof(buf), x, std::chars_format::scientific);
  const char* p = buf;
  const char* end = r.ptr;
  if (*p == '-') {
    out += '-';
    ++p;
  }
  char digits[32];
  int nd = 0;
  while (p < end && *p != 'e') {
    if (*p != '.') digits[nd++] = *p;
    ++p;
  }
  ++p;  // 'e'
  int e = 0;
  std::from_chars(p + (*p == '+' ? 1 : 0), end, e);
  while (nd > 1 && digits[nd - 1] == '0') --nd;  // (shortest output has none; defensive)
  const int kk = e + 1;  // decimal point position: value = 0.DIGITS x 10^kk
  const int k = kk - nd;  // exponent of the last digit
  if (k >= 0 && kk <= 16) {
    out.append(digits, nd);
    out.append((size_t)k, '0');
    out += ".0";
  } else if (kk > 0 && kk <= 16) {
    out.append(digits, kk);
    out += '.';
    out.append(digits + kk, nd - kk);
  } else if (kk > -5 && kk <= 0) {
    out += "0.";
    out.append((size_t)(-kk), '0');
    out.append(digits, nd);
  } else {
    out += digits[0];
    if (nd > 1) {
      out += '.';
      out.append(digits + 1, nd - 1);
    }
    out += 'e';
    char eb[16];
    auto er = std::to_chars(eb, eb + sizeof(eb), kk - 1);
    out.append(eb, er.ptr - eb);
  }
}

void put_str(std::string& out, PyObject* s) {
  Py_ssize_t n = 0;
  const char* u = PyUnicode_AsUTF8AndSize(s, &n);
  if (u == nullptr) throw py::error_already_set();
  out += '"';
  const char* run = u;
  for (Py_ssize_t i = 0; i < n; ++i) {
    const unsigned char c = (unsigned char)u[i];
    if (c >= 0x20 && c != '"' && c != '\\') continue;
    out.append(run, u + i - run);
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default: {
        static const char hex[] = "0123456789abcdef";
        char esc[6] = {'\\', 'u', '0', '0', hex[c >> 4], hex[c & 15]};
        out.append(esc, 6);
      }
    }
    run = u + i + 1;
  }
  out.append(run, u + n - run);
  out += '"';
}

struct Ctx {
  PyObject* plan_of = nullptr;  // callable or null
  PyObject* plans = nullptr;    // dict: type -> plan tuple | None
  PyObject* s_dict = nullptr;   // interned attribute names
  PyObject* s_extra = nullptr;
  PyObject* s_to_obj = nullptr;
};

void put(std::string& out, PyObject* v, int depth, const Ctx& cx);

struct Ref {  // owned reference, released on scope exit (exceptions included)
  PyObject* p;
  explicit Ref(PyObject* o) : p(o) {
    if (p == nullptr) throw py::error_already_set();
  }
  ~Ref() { Py_XDECREF(p); }
};

// a Wire instance by its plan; false when the object has no plan (the caller takes another route)
bool put_wire(std::string& out, PyObject* v, int depth, const Ctx& cx) {
  if (cx.plan_of == nullptr) return false;
  PyObject* tp = (PyObject*)Py_TYPE(v);
  PyObject* plan = PyDict_GetItem(cx.plans, tp);  // borrowed
  if (plan == nullptr) {
    Ref got(PyObject_CallFunctionObjArgs(cx.plan_of, tp, nullptr));
    if (PyDict_SetItem(cx.plans, tp, got.p) < 0) throw py::error_already_set();
    plan = PyDict_GetItem(cx.plans, tp);
  }
  if (plan == Py_False) return false;  // not a Wire
  if (plan == Py_None) {              // its own to_obj()
    Ref o(PyObject_CallMethodObjArgs(v, cx.s_to_obj, nullptr));
    put(out, o.p, depth + 1, cx);
    return true;
  }
  {
    Ref extra(PyObject_GetAttr(v, cx.s_extra));
    if (extra.p != Py_None && PyObject_IsTrue(extra.p)) {
      Ref o(PyObject_CallMethodObjArgs(v, cx.s_to_obj, nullptr));
      put(out, o.p, depth + 1, cx);
      return true;
    }
  }
  Ref d(PyObject_GetAttr(v, cx.s_dict));
  out += '{';
  bool first = true;
  const Py_ssize_t n = PyTuple_GET_SIZE(plan);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* f = PyTuple_GET_ITEM(plan, i);  // (name, key, keep)
    PyObject* x = PyDict_GetItem(d.p, PyTuple_GET_ITEM(f, 0));
    if (x == nullptr) throw TypeErr{};
    if (x == Py_None && PyTuple_GET_ITEM(f, 2) != Py_True) continue;
    if (!first) out += ',';
    first = false;
    put_str(out, PyTuple_GET_ITEM(f, 1));
    out += ':';
    put(out, x, depth + 1, cx);
  }
  out += '}';
  return true;
}

void put(std::string& out, PyObject* v, int depth, const Ctx& cx) {
  if (depth > 512) throw TypeErr{};  // (the Python encoder reports the recursion)
  if (v == Py_None) {
    out += "null";
  } else if (v == Py_True) {
    out += "true";
  } else if (v == Py_False) {
    out += "false";
  } else if (PyUnicode_Check(v)) {
    put_str(out, v);
  } else if (PyLong_Check(v)) {
    int overflow = 0;
    const long long x = PyLong_AsLongLongAndOverflow(v, &overflow);
    if (overflow == 0) {
      if (x == -1 && PyErr_Occurred()) throw py::error_already_set();
      char b[24];
      auto r = std::to_chars(b, b + sizeof(b), x);
      out.append(b, r.ptr - b);
    } else {
      PyObject* s = PyObject_Str(v);
      if (s == nullptr) throw py::error_already_set();
      Py_ssize_t n = 0;
      const char* u = PyUnicode_AsUTF8AndSize(s, &n);
      out.append(u, n);
      Py_DECREF(s);
    }
  } else if (PyFloat_Check(v)) {
    put_f64(out, PyFloat_AS_DOUBLE(v));
  } else if (PyDict_Check(v)) {
    out += '{';
    PyObject *key, *val;
    Py_ssize_t pos = 0;
    bool first = true;
    while (PyDict_Next(v, &pos, &key, &val)) {
      if (!first) out += ',';
      first = false;
      if (PyUnicode_Check(key)) {
        put_str(out, key);
      } else {
        PyObject* s = PyObject_Str(key);
        if (s == nullptr) throw py::error_already_set();
        put_str(out, s);
        Py_DECREF(s);
      }
      out += ':';
      put(out, val, depth + 1, cx);
    }
    out += '}';
  } else if (PyList_Check(v) || PyTuple_Check(v)) {
    out += '[';
    const bool list = PyList_Check(v);
    const Py_ssize_t n = list ? PyList_GET_SIZE(v) : PyTuple_GET_SIZE(v);
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (i) out += ',';
      put(out, list ? PyList_GET_ITEM(v, i) : PyTuple_GET_ITEM(v, i), depth + 1, cx);
    }
    out += ']';
  } else if (!put_wire(out, v, depth, cx)) {
    throw TypeErr{};
  }
}

}  // namespace

void bind_json(py::module_& m) {
  m.def(
      "json_dumps",
      [](py::handle v, py::handle plan_of) -> py::object {
        // type -> plan (types outlive the requests); owned references leaked on purpose: static py objects
        // would be released after the interpreter finalised
        static PyObject* plans = PyDict_New();
        static PyObject* s_dict = PyUnicode_InternFromString("__dict__");
        static PyObject* s_extra = PyUnicode_InternFromString("__pydantic_extra__");
        static PyObject* s_to_obj = PyUnicode_InternFromString("to_obj");
        Ctx cx;
        if (!plan_of.is_none()) {
          cx.plan_of = plan_of.ptr();
          cx.plans = plans;
          cx.s_dict = s_dict;
          cx.s_extra = s_extra;
          cx.s_to_obj = s_to_obj;
        }
        std::string out;
        out.reserve(4096);
        try {
          put(out, v.ptr(), 0, cx);
        } catch (const TypeErr&) {
          throw py::type_error("json_dumps: value outside dict/list/tuple/str/int/float/bool/None");
        }
        PyObject* s = PyUnicode_DecodeUTF8(out.data(), (Py_ssize_t)out.size(), "strict");
        if (s == nullptr) throw py::error_already_set();
        return py::reinterpret_steal<py::object>(s);
      },
      py::arg("v"), py::arg("plan_of") = py::none(),
      "serde_json-compatible compact JSON text of a value tree (floats in ryu form, non-finite as null); "
      "plan_of(cls) -> ((name, key, keep_none), ...) | None (own to_obj) | False (not a wire type)");
  m.def("json_f64", [](double x) {
    std::string out;
    put_f64(out, x);
    return out;
  });
}

}  // namespace lwc
