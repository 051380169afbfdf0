// pybind11 bindings of the host I/O codecs (module streamml._io).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cctype>
#include <cstring>

#include "avro.h"
#include "feed.h"
#include "format.h"
#include "jsonrow.h"
#include "scoreloop.h"
#include "h5.h"
#include "kafka.h"
#include "mqtt.h"

namespace py = pybind11;
using namespace sml;

namespace {

// ---------------------------------------------------------------- HDF5 ------
py::object value_to_py(const h5::Value& v) {
  py::dict d;
  py::list shape;
  for (auto x : v.shape) shape.append(x);
  d["shape"] = shape;
  d["null"] = v.is_null;
  switch (v.kind) {
    case h5::Value::NUMERIC: {
      d["kind"] = "numeric";
      std::string dt = std::string("<") + v.dtype + std::to_string(v.itemsize);
      d["dtype"] = dt;
      d["data"] = py::bytes(v.data);
      break;
    }
    case h5::Value::FIXED_STRING:
      d["kind"] = "fixed_str";
      d["size"] = v.itemsize;
      d["pad"] = v.str_pad;
      d["cset"] = v.cset;
      d["data"] = py::bytes(v.data);
      break;
    case h5::Value::VLEN_STRING: {
      d["kind"] = "vlen_str";
      d["cset"] = v.cset;
      py::list vals;
      for (const auto& s : v.strings) vals.append(py::bytes(s));
      d["values"] = vals;
      break;
    }
  }
  return std::move(d);
}

h5::Value value_from_py(const py::dict& d) {
  h5::Value v;
  const std::string kind = py::str(d["kind"]);
  for (auto x : d["shape"].cast<py::list>()) v.shape.push_back(x.cast<uint64_t>());
  if (kind == "numeric") {
    v.kind = h5::Value::NUMERIC;
    const std::string dt = py::str(d["dtype"]);  // e.g. "<f4"
    if (dt.size() < 3 || dt[0] != '<') throw std::runtime_error("h5: dtype must be little-endian like '<f4'");
    v.dtype = dt[1];
    v.itemsize = std::stoi(dt.substr(2));
    v.data = d["data"].cast<std::string>();
  } else if (kind == "fixed_str") {
    v.kind = h5::Value::FIXED_STRING;
    v.itemsize = d["size"].cast<int>();
    v.str_pad = d.contains("pad") ? d["pad"].cast<int>() : 1;
    v.cset = d.contains("cset") ? d["cset"].cast<int>() : 0;
    v.data = d["data"].cast<std::string>();
  } else if (kind == "vlen_str") {
    v.kind = h5::Value::VLEN_STRING;
    v.cset = d.contains("cset") ? d["cset"].cast<int>() : 1;
    for (auto s : d["values"].cast<py::list>()) v.strings.push_back(s.cast<std::string>());
  } else {
    throw std::runtime_error("h5: unknown value kind " + kind);
  }
  return v;
}

py::dict node_to_py(const h5::Node& n) {
  py::dict d;
  py::dict attrs;
  for (const auto& a : n.attrs) attrs[py::str(a.first)] = value_to_py(a.second);
  d["attrs"] = attrs;
  if (n.is_group) {
    d["type"] = "group";
    py::dict kids;
    for (const auto& c : n.children) kids[py::str(c.first)] = node_to_py(c.second);
    d["children"] = kids;
  } else {
    d["type"] = "dataset";
    d["value"] = value_to_py(n.value);
  }
  return d;
}

h5::Node node_from_py(const py::dict& d) {
  h5::Node n;
  const std::string type = d.contains("type") ? std::string(py::str(d["type"])) : "group";
  n.is_group = type == "group";
  if (d.contains("attrs"))
    for (auto kv : d["attrs"].cast<py::dict>())
      n.attrs.emplace_back(kv.first.cast<std::string>(), value_from_py(kv.second.cast<py::dict>()));
  if (n.is_group) {
    if (d.contains("children"))
      for (auto kv : d["children"].cast<py::dict>())
        n.children.emplace_back(kv.first.cast<std::string>(), node_from_py(kv.second.cast<py::dict>()));
  } else {
    n.value = value_from_py(d["value"].cast<py::dict>());
  }
  return n;
}

// ---------------------------------------------------------------- Avro ------
std::vector<avro::Field> fields_from_py(const py::list& lst) {
  std::vector<avro::Field> out;
  for (auto item : lst) {
    auto t = item.cast<py::tuple>();
    avro::Field f;
    f.name = t[0].cast<std::string>();
    f.kind = t[1].cast<int>();
    f.null_branch = t[2].cast<int>();
    f.fixed_size = t.size() > 3 ? t[3].cast<int>() : 0;
    f.n_symbols = t.size() > 4 ? t[4].cast<int>() : 0;
    out.push_back(f);
  }
  return out;
}

// failure_occurred-style label code of a text value: "false" -> 0, "true" -> 1, else 2
// (case-insensitive, surrounding whitespace ignored) -- the stream's LABEL_* codes
uint8_t label_code(const std::string& v) {
  size_t a = 0, e = v.size();
  while (a < e && std::isspace((unsigned char)v[a])) ++a;
  while (e > a && std::isspace((unsigned char)v[e - 1])) --e;
  auto eq = [&](const char* w, size_t n) {
    if (e - a != n) return false;
    for (size_t i = 0; i < n; ++i)
      if (std::tolower((unsigned char)v[a + i]) != w[i]) return false;
    return true;
  };
  return eq("false", 5) ? 0 : eq("true", 4) ? 1 : 2;
}

py::dict batch_to_py(avro::DecodedBatch& b, bool with_text = true) {
  py::dict d;
  const size_t n = b.n, k = b.n_numeric;
  py::array_t<float> num({n, k});
  if (n * k) std::memcpy(num.mutable_data(), b.numeric.data(), n * k * sizeof(float));
  d["numeric"] = num;
  if (!b.numeric64.empty()) {
    py::array_t<double> num64({n, k});
    std::memcpy(num64.mutable_data(), b.numeric64.data(), n * k * sizeof(double));
    d["numeric64"] = num64;
  }
  py::array_t<uint8_t> nul({n, k});
  if (n * k) std::memcpy(nul.mutable_data(), b.null_mask.data(), n * k);
  d["null"] = nul;
  py::list text, tnull, tcodes;
  for (size_t c = 0; c < b.text.size(); ++c) {
    if (with_text) {
      py::list col;
      for (auto& s : b.text[c]) col.append(py::bytes(s));
      text.append(col);
    }
    py::array_t<uint8_t> tn(n), tc(n);
    if (n) std::memcpy(tn.mutable_data(), b.text_null[c].data(), n);
    uint8_t* pc = tc.mutable_data();
    for (py::ssize_t i = 0; i < n; ++i) pc[i] = b.text_null[c][(size_t)i] ? 2 : label_code(b.text[c][(size_t)i]);
    tnull.append(tn);
    tcodes.append(tc);
  }
  d["text"] = text;
  d["text_null"] = tnull;
  d["text_codes"] = tcodes;   // per text column: LABEL_FALSE / LABEL_TRUE / LABEL_MISSING codes
  py::array_t<int32_t> sid(n);
  if (n) std::memcpy(sid.mutable_data(), b.schema_id.data(), n * 4);
  d["schema_id"] = sid;
  py::array_t<uint8_t> ok(n);
  if (n) std::memcpy(ok.mutable_data(), b.ok.data(), n);
  d["ok"] = ok;
  d["n_errors"] = b.n_errors;
  return d;
}

py::dict fetch_to_py(kafka::FetchResult& r) {
  py::dict d;
  d["values"] = py::bytes(r.values);
  py::array_t<int64_t> vo(r.value_offsets.size());
  std::memcpy(vo.mutable_data(), r.value_offsets.data(), r.value_offsets.size() * 8);
  d["value_offsets"] = vo;
  py::array_t<int64_t> off(r.offsets.size());
  if (!r.offsets.empty()) std::memcpy(off.mutable_data(), r.offsets.data(), r.offsets.size() * 8);
  d["offsets"] = off;
  py::array_t<int64_t> ts(r.timestamps.size());
  if (!r.timestamps.empty()) std::memcpy(ts.mutable_data(), r.timestamps.data(), r.timestamps.size() * 8);
  d["timestamps"] = ts;
  py::list keys;
  for (auto& k : r.keys) keys.append(py::bytes(k));
  d["keys"] = keys;
  d["high_watermark"] = r.high_watermark;
  return d;
}

std::vector<kafka::Record> records_from_py(const py::list& values, const py::object& keys, const py::object& ts) {
  std::vector<kafka::Record> recs(values.size());
  py::list kl = keys.is_none() ? py::list() : keys.cast<py::list>();
  py::list tl = ts.is_none() ? py::list() : ts.cast<py::list>();
  for (size_t i = 0; i < recs.size(); ++i) {
    recs[i].value = values[i].cast<std::string>();
    if (!keys.is_none() && !kl[i].is_none()) {
      recs[i].key = kl[i].cast<std::string>();
      recs[i].key_null = false;
    }
    recs[i].timestamp = ts.is_none() ? 0 : tl[i].cast<int64_t>();
  }
  return recs;
}

}  // namespace

PYBIND11_MODULE(_io, m) {
  m.doc() = "streamml host I/O: HDF5, Avro/Confluent, Kafka wire protocol";

  py::register_exception<h5::Error>(m, "H5Error");
  py::register_exception<avro::Error>(m, "AvroError");
  // KafkaError carries the protocol error code as `.code` (1 = OFFSET_OUT_OF_RANGE: the consumer's
  // position was deleted by retention -> auto.offset.reset)
  static py::exception<kafka::Error> kafka_exc(m, "KafkaError");
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const kafka::Error& e) {
      py::object cls = py::reinterpret_borrow<py::object>(kafka_exc.ptr());
      py::object inst = cls(py::str(e.what()));
      inst.attr("code") = e.code;
      PyErr_SetObject(kafka_exc.ptr(), inst.ptr());
    }
  });

  // HDF5
  m.def("h5_read", [](const std::string& path) { return node_to_py(h5::read_file(path)); }, py::arg("path"));
  m.def("h5_read_bytes", [](const py::bytes& b) { return node_to_py(h5::read_bytes(b.cast<std::string>())); },
        py::arg("data"));
  m.def("h5_write", [](const std::string& path, const py::dict& root) { h5::write_file(path, node_from_py(root)); },
        py::arg("path"), py::arg("root"));
  m.def("h5_write_bytes", [](const py::dict& root) { return py::bytes(h5::write_bytes(node_from_py(root))); },
        py::arg("root"));

  // Avro
  py::class_<avro::Codec>(m, "AvroCodec")
      .def(py::init([](const py::list& f) { return new avro::Codec(fields_from_py(f)); }), py::arg("fields"))
      .def_property_readonly("n_numeric", &avro::Codec::n_numeric)
      .def_property_readonly("n_text", &avro::Codec::n_text)
      .def(
          "decode",
          [](const avro::Codec& c, const py::bytes& buf, py::array_t<int64_t, py::array::c_style> offsets,
             bool framing, bool strict, bool want_f64) {
            std::string_view sv = buf;  // no copy
            const size_t n = offsets.size() ? (size_t)offsets.size() - 1 : 0;
            avro::DecodedBatch b;
            {
              py::gil_scoped_release rel;
              b = c.decode(reinterpret_cast<const uint8_t*>(sv.data()), sv.size(), offsets.data(), n, framing, strict,
                           want_f64);
            }
            return batch_to_py(b);
          },
          py::arg("buf"), py::arg("offsets"), py::arg("framing") = true, py::arg("strict") = false,
          py::arg("want_f64") = false)
      .def(
          "encode",
          [](const avro::Codec& c, py::array_t<double, py::array::c_style | py::array::forcecast> numeric,
             py::object null_mask, const py::list& text, py::object text_null, bool framing, int32_t schema_id) {
            const size_t n = numeric.ndim() ? (size_t)numeric.shape(0) : 0;
            if (numeric.ndim() != 2 || (size_t)numeric.shape(1) != c.n_numeric())
              throw avro::Error("avro encode: numeric must be [n, n_numeric]");
            std::vector<uint8_t> nm;
            if (!null_mask.is_none()) {
              auto a = null_mask.cast<py::array_t<uint8_t, py::array::c_style | py::array::forcecast>>();
              nm.assign(a.data(), a.data() + a.size());
            }
            std::vector<std::vector<std::string>> tx;
            for (auto col : text) {
              std::vector<std::string> v;
              for (auto s : col.cast<py::list>()) v.push_back(s.cast<std::string>());
              tx.push_back(std::move(v));
            }
            std::vector<std::vector<uint8_t>> tn;
            if (!text_null.is_none())
              for (auto col : text_null.cast<py::list>()) {
                auto a = col.cast<py::array_t<uint8_t, py::array::c_style | py::array::forcecast>>();
                tn.emplace_back(a.data(), a.data() + a.size());
              }
            std::string out;
            std::vector<int64_t> offs;
            c.encode(numeric.data(), nm.empty() ? nullptr : nm.data(), tx, tn, n, framing, schema_id, out, offs);
            py::array_t<int64_t> po(offs.size());
            std::memcpy(po.mutable_data(), offs.data(), offs.size() * 8);
            return py::make_tuple(py::bytes(out), po);
          },
          py::arg("numeric"), py::arg("null_mask") = py::none(), py::arg("text") = py::list(),
          py::arg("text_null") = py::none(), py::arg("framing") = true, py::arg("schema_id") = 1);

  // Kafka
  m.def("crc32c", [](const py::bytes& b) {
    std::string_view s = b;
    return kafka::crc32c(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  py::class_<kafka::Client>(m, "KafkaClient")
      .def(py::init([](const std::string& bootstrap, const std::string& client_id, const std::string& mech,
                       const std::string& user, const std::string& pw, int timeout_ms) {
             kafka::ClientConfig c;
             c.client_id = client_id;
             c.sasl_mechanism = mech;
             c.sasl_username = user;
             c.sasl_password = pw;
             c.timeout_ms = timeout_ms;
             return new kafka::Client(bootstrap, c);
           }),
           py::arg("bootstrap"), py::arg("client_id") = "streamml", py::arg("sasl_mechanism") = "",
           py::arg("sasl_username") = "", py::arg("sasl_password") = "", py::arg("timeout_ms") = 30000)
      .def("partitions", [](kafka::Client& c) {
        py::gil_scoped_release rel;
        return c.partitions();
      })
      .def("list_offset",
           [](kafka::Client& c, const std::string& t, int p, int64_t time) {
             py::gil_scoped_release rel;
             return c.list_offset(t, p, time);
           },
           py::arg("topic"), py::arg("partition"), py::arg("time"))
      .def("fetch",
           [](kafka::Client& c, const std::string& t, int p, int64_t off, int32_t max_bytes, int32_t wait) {
             kafka::FetchResult r;
             {
               py::gil_scoped_release rel;
               r = c.fetch(t, p, off, max_bytes, wait);
             }
             return fetch_to_py(r);
           },
           py::arg("topic"), py::arg("partition"), py::arg("offset"), py::arg("max_bytes") = 1 << 20,
           py::arg("max_wait_ms") = 100)
      .def("fetch_decode",
           [](kafka::Client& c, const avro::Codec& codec, const std::string& t, int p, int64_t off,
              int32_t max_bytes, int32_t wait, bool framing, bool with_text, bool str_keys) {
             kafka::FetchResult r;
             avro::DecodedBatch b;
             {
               py::gil_scoped_release rel;
               r = c.fetch(t, p, off, max_bytes, wait);
               b = codec.decode(reinterpret_cast<const uint8_t*>(r.values.data()), r.values.size(),
                                r.value_offsets.data(), r.size(), framing, false, false);
             }
             py::dict d = batch_to_py(b, with_text);
             py::array_t<int64_t> offs(r.offsets.size());
             if (!r.offsets.empty()) std::memcpy(offs.mutable_data(), r.offsets.data(), r.offsets.size() * 8);
             d["offsets"] = offs;
             py::list keys;
             if (str_keys) {
               for (auto& k : r.keys) keys.append(py::reinterpret_steal<py::object>(
                   PyUnicode_DecodeUTF8(k.data(), (py::ssize_t)k.size(), "replace")));
             } else {
               for (auto& k : r.keys) keys.append(py::bytes(k));
             }
             d["keys"] = keys;
             d["high_watermark"] = r.high_watermark;
             d["bytes"] = r.values.size();
             return d;
           },
           py::arg("codec"), py::arg("topic"), py::arg("partition"), py::arg("offset"),
           py::arg("max_bytes") = 1 << 20, py::arg("max_wait_ms") = 100, py::arg("framing") = true,
           py::arg("with_text") = true, py::arg("str_keys") = false)
      .def("produce",
           [](kafka::Client& c, const std::string& t, int p, const py::list& values, py::object keys, py::object ts,
              int acks) {
             auto recs = records_from_py(values, keys, ts);
             py::gil_scoped_release rel;
             return c.produce(t, p, recs, (int16_t)acks);
           },
           py::arg("topic"), py::arg("partition"), py::arg("values"), py::arg("keys") = py::none(),
           py::arg("timestamps") = py::none(), py::arg("acks") = 1)
      .def("commit",
           [](kafka::Client& c, const std::string& g, const std::string& t, int p, int64_t off) {
             py::gil_scoped_release rel;
             c.commit(g, t, p, off);
           })
      .def("committed",
           [](kafka::Client& c, const std::string& g, const std::string& t, int p) {
             py::gil_scoped_release rel;
             return c.committed(g, t, p);
           })
      .def_property_readonly("bytes_received", &kafka::Client::bytes_received);

  // native ingest feed: worker threads decode Kafka records straight into caller slabs
  // ---- low-latency streaming scorer (scoreloop.h) ----
  struct EchoScorer {   // CPU stand-in for the GPU scorer (tests): score = mean(x^2), recon = x / 2
    SmlScorerApi api{};  // keyed (nkeys > 0): score = the row's key slot, flag 2 on a slot's first event
    float thr;
    std::vector<uint8_t> seen;
    static int infer(void* ctx, const float* rows, int k, float* scores, uint32_t* flags, float* recon, double) {
      auto* self = static_cast<EchoScorer*>(ctx);
      const int D = self->api.dim;
      for (int i = 0; i < k; ++i) {
        float s = 0.0f;
        for (int j = 0; j < D; ++j) {
          const float x = rows[(size_t)i * D + j];
          s += x * x;
          if (recon) recon[(size_t)i * D + j] = 0.5f * x;
        }
        scores[i] = s / (float)D;
        flags[i] = scores[i] > self->thr ? 1u : 0u;
      }
      return 0;
    }
    static int infer_keyed(void* ctx, const float* rows, const uint32_t* keys, int k, float* scores,
                           uint32_t* flags, float* recon, double t) {
      auto* self = static_cast<EchoScorer*>(ctx);
      infer(ctx, rows, k, scores, flags, recon, t);
      for (int i = 0; i < k; ++i) {
        if ((int64_t)keys[i] >= self->api.nkeys) return 1;
        scores[i] = (float)keys[i];
        flags[i] = self->seen[keys[i]] ? 0u : 2u;
        self->seen[keys[i]] = 1;
      }
      return 0;
    }
  };
  py::class_<EchoScorer>(m, "EchoScorer")
      .def(py::init([](int dim, float threshold, int64_t nkeys) {
             auto* e = new EchoScorer();
             e->api.version = SML_SCORER_API_VERSION;
             e->api.dim = dim;
             e->api.ctx = e;
             e->api.infer = &EchoScorer::infer;
             e->api.last_error = nullptr;
             e->api.nkeys = nkeys;
             e->api.infer_keyed = nkeys > 0 ? &EchoScorer::infer_keyed : nullptr;
             e->seen.assign((size_t)std::max<int64_t>(nkeys, 0), 0);
             e->thr = threshold;
             return e;
           }),
           py::arg("dim"), py::arg("threshold") = 5.0f, py::arg("nkeys") = 0)
      .def("c_api", [](EchoScorer& e) { return reinterpret_cast<uintptr_t>(&e.api); });
  m.def("key_share_hash", [](py::bytes key) {
    const std::string k = key;
    return serve::key_share_hash(reinterpret_cast<const uint8_t*>(k.data()), (int64_t)k.size());
  }, "FNV-1a 64 >> 32 of a record key (the serving loop's key-share hash; kafka/assign.py key_hash)");
  py::class_<serve::ScoreLoop>(m, "ScoreLoop")
      .def(py::init([](const std::string& bootstrap, const std::string& client_id, const std::string& mech,
                       const std::string& user, const std::string& pw, int timeout_ms, const py::list& fields,
                       const std::string& topic, const std::string& result_topic, const std::string& group,
                       std::vector<int> partitions, std::vector<int64_t> starts, std::vector<int> result_partitions,
                       std::vector<int> feature_fields, bool framing, bool emit_recon, int max_batch,
                       int32_t max_bytes, int32_t max_wait_ms, double commit_interval_s, bool record_latency,
                       uintptr_t api, int spin_us, std::vector<std::pair<std::string, int>> json_columns,
                       const std::string& json_stamp, std::vector<std::pair<uint64_t, uint64_t>> hash_ranges,
                       int offset_reset) {
             kafka::ClientConfig c;
             c.client_id = client_id;
             c.sasl_mechanism = mech;
             c.sasl_username = user;
             c.sasl_password = pw;
             c.timeout_ms = timeout_ms;
             c.spin_us = spin_us;
             serve::LoopConfig lc;
             lc.topic = topic;
             lc.result_topic = result_topic;
             lc.group = group;
             lc.partitions = std::move(partitions);
             lc.starts = std::move(starts);
             lc.result_partitions = std::move(result_partitions);
             lc.feature_fields = std::move(feature_fields);
             lc.framing = framing;
             lc.emit_recon = emit_recon;
             lc.max_batch = max_batch;
             lc.max_bytes = max_bytes;
             lc.max_wait_ms = max_wait_ms;
             lc.commit_interval_s = commit_interval_s;
             lc.record_latency = record_latency;
             lc.json_columns = std::move(json_columns);
             lc.json_stamp = json_stamp;
             lc.hash_ranges = std::move(hash_ranges);
             lc.offset_reset = offset_reset;
             return new serve::ScoreLoop(bootstrap, c, fields_from_py(fields), lc,
                                         reinterpret_cast<const SmlScorerApi*>(api));
           }),
           py::arg("bootstrap"), py::arg("client_id"), py::arg("sasl_mechanism"), py::arg("sasl_username"),
           py::arg("sasl_password"), py::arg("timeout_ms"), py::arg("fields"), py::arg("topic"),
           py::arg("result_topic"), py::arg("group"), py::arg("partitions"), py::arg("starts"),
           py::arg("result_partitions"), py::arg("feature_fields"), py::arg("framing"), py::arg("emit_recon"),
           py::arg("max_batch"), py::arg("max_bytes"), py::arg("max_wait_ms"), py::arg("commit_interval_s"),
           py::arg("record_latency"), py::arg("scorer_api"), py::arg("spin_us") = 0,
           py::arg("json_columns") = std::vector<std::pair<std::string, int>>{}, py::arg("json_stamp") = "",
           py::arg("hash_ranges") = std::vector<std::pair<uint64_t, uint64_t>>{}, py::arg("offset_reset") = 0)
      .def("run",
           [](serve::ScoreLoop& l, int64_t max_events, double idle_timeout_s) {
             serve::LoopStats st;
             {
               py::gil_scoped_release nogil;
               st = l.run(max_events, idle_timeout_s);
             }
             py::dict d;
             d["events"] = st.events;
             d["anomalies"] = st.anomalies;
             d["skipped"] = st.skipped;
             d["batches"] = st.batches;
             d["fetches"] = st.fetches;
             d["empty_fetches"] = st.empty_fetches;
             d["commits"] = st.commits;
             d["fetch_s"] = st.fetch_s;
             d["decode_s"] = st.decode_s;
             d["score_s"] = st.score_s;
             d["format_s"] = st.format_s;
             d["produce_s"] = st.produce_s;
             d["commit_s"] = st.commit_s;
             d["wall_s"] = st.wall_s;
             d["keys"] = st.keys;
             d["foreign"] = st.foreign;
             d["keys_dropped"] = st.keys_dropped;
             d["reset_skipped"] = st.reset_skipped;
             return d;
           },
           py::arg("max_events") = 0, py::arg("idle_timeout_s") = -1.0)
      .def("stop", &serve::ScoreLoop::stop)
      .def("positions", &serve::ScoreLoop::positions)
      .def("latency_bytes", &serve::ScoreLoop::latency_bytes)
      .def("latency_records", [](serve::ScoreLoop& l) {
        const auto& v = l.latency_records();
        constexpr int C = serve::ScoreLoop::kLatCols;
        py::array_t<int64_t> a(std::vector<ssize_t>{(ssize_t)(v.size() / C), C});
        std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(int64_t));
        return a;
      });
  m.def("paced_produce",
        [](const std::string& bootstrap, const std::string& topic, int partition, const py::bytes& values,
           std::vector<int64_t> offs, py::object keys, double qps, int spin_us) {
          std::string vals = values;
          std::vector<std::string> ks;
          if (!keys.is_none())
            for (auto h : keys.cast<py::list>()) ks.push_back(py::isinstance<py::bytes>(h) ? h.cast<std::string>()
                                                                                     : py::str(h).cast<std::string>());
          std::vector<int64_t> sent;
          {
            py::gil_scoped_release nogil;
            kafka::ClientConfig c;
            c.spin_us = spin_us;
            sent = serve::paced_produce(bootstrap, c, topic, partition, vals, offs, ks, qps);
          }
          return py::array_t<int64_t>((ssize_t)sent.size(), sent.data());
        },
        py::arg("bootstrap"), py::arg("topic"), py::arg("partition"), py::arg("values"), py::arg("offsets"),
        py::arg("keys") = py::none(), py::arg("qps") = 10000.0, py::arg("spin_us") = 0,
        "append records one produce request each at `qps`; -> steady-clock send time (ns) per record");
  m.def("steady_ns", &serve::steady_ns);

  // ---- JSON car-event records (jsonrow.h): the bridge's sensor-data / KSQL SENSOR_DATA_S ----
  m.def("json_canonical", &jsonrow::canonical, py::arg("key"));
  m.def("json_rows",
        [](const py::bytes& values, std::vector<int64_t> offs, std::vector<std::pair<std::string, int>> columns,
           const std::string& label_key, const std::string& stamp_key) {
          const jsonrow::Plan plan(columns, label_key, stamp_key);
          std::string_view v(values);
          const ssize_t n = offs.empty() ? 0 : (ssize_t)offs.size() - 1;
          const int F = plan.width();
          py::array_t<float> rows(std::vector<ssize_t>{n, F});
          py::array_t<uint8_t> labels(n), ok(n);
          py::array_t<int64_t> stamps(n);
          float* pr = rows.mutable_data();
          uint8_t* pl = labels.mutable_data();
          uint8_t* po = ok.mutable_data();
          int64_t* ps = stamps.mutable_data();
          {
            py::gil_scoped_release nogil;
            for (ssize_t i = 0; i < n; ++i) {
              const int64_t a = offs[(size_t)i], b = offs[(size_t)i + 1];
              if (a < 0 || b < a || (size_t)b > v.size()) throw std::out_of_range("json_rows: bad offsets");
              po[i] = plan.decode(reinterpret_cast<const uint8_t*>(v.data()) + a, (size_t)(b - a), pr + i * F,
                                  pl + i, ps + i)
                          ? 1
                          : 0;
            }
          }
          return py::make_tuple(rows, labels, stamps, ok);
        },
        py::arg("values"), py::arg("offsets"), py::arg("columns"), py::arg("label_key") = "",
        py::arg("stamp_key") = "",
        "JSON records values[offs[i]:offs[i+1]] -> (rows [n, F] float32 (NaN = missing), label codes, stamps, ok)");

  // ---- result-record formatting (format.h) ----
  m.def("array2string_f32",
        [](py::array_t<float, py::array::c_style | py::array::forcecast> a) {
          std::string out;
          fmt::array2string_f32(a.data(), (int)a.size(), out);
          return out;
        },
        "numpy.array2string of a 1-D float32 array (default options), in C++");
  m.def("json_float", [](double v) {
    std::string out;
    fmt::py_float_repr(v, out);
    return out;
  });
  m.def("score_records",
        [](py::object keys, int partition, py::array_t<int64_t, py::array::c_style | py::array::forcecast> offsets,
           py::array_t<float, py::array::c_style | py::array::forcecast> scores,
           py::array_t<uint8_t, py::array::c_style | py::array::forcecast> flags, py::object recon) {
          const int64_t k = scores.size();
          if (offsets.size() != k || flags.size() != k) throw std::invalid_argument("score_records: length mismatch");
          std::vector<std::string> ks;
          std::vector<char> knull((size_t)k, 1);
          if (!keys.is_none()) {
            py::list kl = keys;
            if ((int64_t)kl.size() != k) throw std::invalid_argument("score_records: keys length mismatch");
            ks.resize((size_t)k);
            for (int64_t i = 0; i < k; ++i) {
              py::handle h = kl[(size_t)i];
              if (h.is_none()) continue;
              knull[(size_t)i] = 0;
              if (py::isinstance<py::bytes>(h)) ks[(size_t)i] = h.cast<std::string>();
              else ks[(size_t)i] = py::str(h).cast<std::string>();
            }
          }
          py::array_t<float, py::array::c_style | py::array::forcecast> rec;
          int D = 0;
          if (!recon.is_none()) {
            rec = recon.cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
            if (rec.ndim() != 2 || rec.shape(0) != k) throw std::invalid_argument("score_records: recon must be [k, D]");
            D = (int)rec.shape(1);
          }
          std::vector<std::string> out((size_t)k);
          {
            py::gil_scoped_release nogil;
            for (int64_t i = 0; i < k; ++i) {
              const bool kn = ks.empty() || knull[(size_t)i];
              fmt::score_record_json(kn ? nullptr : reinterpret_cast<const uint8_t*>(ks[(size_t)i].data()),
                                     kn ? -1 : (int64_t)ks[(size_t)i].size(), partition, offsets.data()[i],
                                     scores.data()[i], flags.data()[i] != 0, D ? rec.data() + i * D : nullptr, D,
                                     out[(size_t)i]);
            }
          }
          py::list res;
          for (auto& r : out) res.append(py::bytes(r));
          return res;
        },
        py::arg("keys"), py::arg("partition"), py::arg("offsets"), py::arg("scores"), py::arg("flags"),
        py::arg("recon") = py::none(),
        "the serve result records (json.dumps of {car, partition, offset, score, anomaly[, reconstruction]}) in C++");
  m.def("label_code", [](const py::bytes& b) {
    std::string_view s = b;
    return (int)feed::label_code(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  py::class_<feed::Feed>(m, "KafkaFeed")
      .def(py::init([](const std::string& bootstrap, const std::string& client_id, const std::string& mech,
                       const std::string& user, const std::string& pw, int timeout_ms, const py::list& fields,
                       std::vector<int> feature_fields, int label_field, int keep_label, bool framing,
                       int32_t max_bytes, int32_t max_wait_ms, int workers, double idle_timeout_s,
                       const std::vector<std::tuple<std::string, int, int64_t, int64_t>>& parts, bool check_crcs,
                       int offset_reset) {
             kafka::ClientConfig c;
             c.client_id = client_id;
             c.sasl_mechanism = mech;
             c.sasl_username = user;
             c.sasl_password = pw;
             c.timeout_ms = timeout_ms;
             feed::FeedConfig fc;
             fc.feature_fields = std::move(feature_fields);
             fc.label_field = label_field;
             fc.keep_label = keep_label;
             fc.framing = framing;
             fc.max_bytes = max_bytes;
             fc.max_wait_ms = max_wait_ms;
             fc.workers = workers;
             fc.idle_timeout_s = idle_timeout_s;
             fc.check_crcs = check_crcs;
             fc.offset_reset = offset_reset;
             std::vector<feed::PartSpec> ps;
             for (const auto& t : parts) ps.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t)});
             return new feed::Feed(bootstrap, c, fields_from_py(fields), fc, ps);
           }),
           py::arg("bootstrap"), py::arg("client_id"), py::arg("sasl_mechanism"), py::arg("sasl_username"),
           py::arg("sasl_password"), py::arg("timeout_ms"), py::arg("fields"), py::arg("feature_fields"),
           py::arg("label_field"), py::arg("keep_label"), py::arg("framing"), py::arg("max_bytes"),
           py::arg("max_wait_ms"), py::arg("workers"), py::arg("idle_timeout_s"), py::arg("parts"),
           py::arg("check_crcs") = false, py::arg("offset_reset") = 0)
      .def("start",
           [](feed::Feed& f, const std::vector<uint64_t>& slabs, int64_t cap) {
             std::vector<uintptr_t> v(slabs.begin(), slabs.end());
             f.start(v, cap);
           },
           py::arg("slabs"), py::arg("cap_rows"))
      .def("start_staged",   // pre-staged record values -> the slabs (the caller keeps buf / offsets alive)
           [](feed::Feed& f, const std::vector<uint64_t>& slabs, int64_t cap, py::buffer buf,
              py::array_t<int64_t, py::array::c_style> offs, int workers) {
             py::buffer_info bi = buf.request();
             const int64_t n = (int64_t)offs.size() - 1;
             if (n < 0 || (n > 0 && offs.at(n) > (int64_t)bi.size * (int64_t)bi.itemsize))
               throw std::invalid_argument("start_staged: offsets past the buffer");
             std::vector<uintptr_t> v(slabs.begin(), slabs.end());
             f.start_staged(v, cap, static_cast<const uint8_t*>(bi.ptr), offs.data(), n, workers);
           },
           py::arg("slabs"), py::arg("cap_rows"), py::arg("buf"), py::arg("offsets"), py::arg("workers"))
      .def("pop",
           [](feed::Feed& f, int timeout_ms) {
             int slab = -1;
             int64_t rows = 0;
             int r;
             {
               py::gil_scoped_release rel;
               r = f.pop(slab, rows, timeout_ms);
             }
             return py::make_tuple(r, slab, rows);
           },
           py::arg("timeout_ms") = -1)
      .def("recycle", &feed::Feed::recycle, py::arg("slab"))
      .def("stop",
           [](feed::Feed& f) {
             py::gil_scoped_release rel;
             f.stop();
           })
      .def("decode_throughput",   // pre-staged values -> (best rows/s, rows kept per pass); no broker
           [](const feed::Feed& f, py::buffer buf, py::array_t<int64_t, py::array::c_style | py::array::forcecast> offs,
              int workers, int repeats) {
             py::buffer_info bi = buf.request();
             const int64_t n = (int64_t)offs.size() - 1;
             if (n < 1 || offs.at(n) > (int64_t)bi.size * (int64_t)bi.itemsize)
               throw std::invalid_argument("decode_throughput: offsets past the buffer");
             int64_t rows = 0;
             double r;
             {
               py::gil_scoped_release rel;
               r = f.decode_throughput(static_cast<const uint8_t*>(bi.ptr), offs.data(), n, workers, repeats, &rows);
             }
             return py::make_tuple(r, rows);
           },
           py::arg("buf"), py::arg("offsets"), py::arg("workers"), py::arg("repeats") = 3)
      .def("decode_row",   // one framed Avro value -> (ok, projected row, label code); tests / debugging
           [](const feed::Feed& f, const py::bytes& value) {
             const std::string v = value;
             std::vector<float> row((size_t)f.features(), 0.f);
             uint8_t lab = 0;
             const bool ok = f.decode_row(reinterpret_cast<const uint8_t*>(v.data()), v.size(), row.data(), &lab);
             return py::make_tuple(ok, row, (int)lab);
           }, py::arg("value"))
      .def_property_readonly("fast_plan", &feed::Feed::fast_plan)
      .def("positions", &feed::Feed::positions)
      .def("slab_marks", &feed::Feed::slab_marks, py::arg("slab"))
      .def_property_readonly("features", &feed::Feed::features)
      .def("stats", [](const feed::Feed& f) {
        const feed::Stats s = f.stats();
        py::dict d;
        d["records"] = s.records;
        d["rows"] = s.rows;
        d["dropped"] = s.dropped;
        d["errors"] = s.errors;
        d["bytes"] = s.bytes;
        d["fetches"] = s.fetches;
        d["slabs"] = s.slabs;
        d["fetch_s"] = s.fetch_s;
        d["decode_s"] = s.decode_s;
        d["wait_slab_s"] = s.wait_slab_s;
        d["reset_skipped"] = s.reset_skipped;
        return d;
      });

  py::class_<kafka::Broker>(m, "KafkaBroker")
      .def(py::init([](int port, const std::string& user, const std::string& pw, int64_t retention,
                       int64_t message_max_bytes, int64_t retention_ms, int64_t retention_bytes, int check_ms) {
             kafka::BrokerConfig c;
             c.port = port;
             c.sasl_username = user;
             c.sasl_password = pw;
             c.retention_records = retention;
             c.message_max_bytes = message_max_bytes;
             c.retention_ms = retention_ms;
             c.retention_bytes = retention_bytes;
             c.retention_check_ms = check_ms;
             return new kafka::Broker(c);
           }),
           py::arg("port") = 0, py::arg("sasl_username") = "", py::arg("sasl_password") = "",
           py::arg("retention_records") = -1, py::arg("message_max_bytes") = 1048588, py::arg("retention_ms") = -1,
           py::arg("retention_bytes") = -1, py::arg("retention_check_ms") = 1000)
      .def_property_readonly("port", &kafka::Broker::port)
      .def("create_topic", &kafka::Broker::create_topic, py::arg("name"), py::arg("partitions"),
           py::arg("retention_ms") = -2, py::arg("retention_bytes") = -2)
      .def("enforce_retention",
           [](kafka::Broker& b) {
             py::gil_scoped_release rel;
             return b.enforce_retention();
           })
      .def_property_readonly("deleted_segments", &kafka::Broker::deleted_segments)
      .def_property_readonly("deleted_records", &kafka::Broker::deleted_records)
      .def("log_bytes", &kafka::Broker::log_bytes)
      .def("log_segments", &kafka::Broker::log_segments)
      .def("append",
           [](kafka::Broker& b, const std::string& t, int p, const py::list& values, py::object keys,
              py::object ts) { return b.append(t, p, records_from_py(values, keys, ts)); },
           py::arg("topic"), py::arg("partition"), py::arg("values"), py::arg("keys") = py::none(),
           py::arg("timestamps") = py::none())
      .def("append_buffer",
           [](kafka::Broker& b, const std::string& t, int p, const py::bytes& buf,
              py::array_t<int64_t, py::array::c_style> offsets, int64_t ts0) {
             std::string_view sv = buf;
             std::vector<kafka::Record> recs((size_t)std::max<py::ssize_t>(0, offsets.size() - 1));
             for (size_t i = 0; i < recs.size(); ++i) {
               recs[i].value.assign(sv.data() + offsets.data()[i], (size_t)(offsets.data()[i + 1] - offsets.data()[i]));
               recs[i].timestamp = ts0;
             }
             py::gil_scoped_release rel;
             return b.append(t, p, recs);
           },
           py::arg("topic"), py::arg("partition"), py::arg("buf"), py::arg("offsets"), py::arg("timestamp") = 0)
      .def("end_offset", &kafka::Broker::end_offset)
      .def("start_offset", &kafka::Broker::start_offset)
      .def("read",
           [](kafka::Broker& b, const std::string& t, int p, int64_t off, size_t maxn) {
             auto recs = b.read(t, p, off, maxn);
             py::list out;
             for (auto& r : recs) out.append(py::make_tuple(r.offset, py::bytes(r.key), py::bytes(r.value)));
             return out;
           })
      .def("set_faults", &kafka::Broker::set_faults, py::arg("fail_every") = 0, py::arg("delay_ms") = 0)
      .def("set_thread_cpus", &kafka::Broker::set_thread_cpus, py::arg("cpus"),
           "CPUs for connection threads accepted from now on (empty: unpinned)")
      .def("set_spin_us", &kafka::Broker::set_spin_us, py::arg("us"),
           "low-latency mode: connection threads and empty long polls busy-wait this long first")
      .def("record_append_times", &kafka::Broker::record_append_times, py::arg("on") = true)
      .def("append_times",
           [](kafka::Broker& b, const std::string& t, int p, int64_t start, int64_t count) {
             const auto v = b.append_times(t, p, start, count);
             return py::array_t<int64_t>((ssize_t)v.size(), v.data());
           },
           py::arg("topic"), py::arg("partition"), py::arg("start"), py::arg("count"),
           "steady-clock append time (ns) per offset, -1 where not recorded")
      .def_property_readonly("fetch_count", &kafka::Broker::fetch_count)
      .def_property_readonly("injected_failures", &kafka::Broker::injected_failures)
      .def("stop", [](kafka::Broker& b) {
        py::gil_scoped_release rel;
        b.stop();
      });

  // MQTT (broker + Kafka bridge, client, device simulator)
  m.def("mqtt_topic_matches", &mqtt::topic_matches, py::arg("filter"), py::arg("topic"));
  m.def("mqtt_valid_filter", &mqtt::valid_filter, py::arg("filter"));
  m.def("kafka_partition", &mqtt::kafka_partition, py::arg("key"), py::arg("partitions"),
        "Kafka default partitioner: murmur2(key) & 0x7fffffff % partitions");
  m.def("murmur2", &mqtt::murmur2, py::arg("key"));
  m.def("mqtt_encode_publish", [](const std::string& topic, const py::bytes& payload, int qos, bool retain,
                                  int packet_id, int version) {
    mqtt::Message msg;
    msg.topic = topic;
    msg.payload = payload;
    msg.qos = qos;
    msg.retain = retain;
    msg.packet_id = (uint16_t)packet_id;
    return py::bytes(mqtt::encode_publish(msg, version));
  }, py::arg("topic"), py::arg("payload"), py::arg("qos") = 0, py::arg("retain") = false,
        py::arg("packet_id") = 0, py::arg("version") = 5);
  m.def("mqtt_parse_packet", [](const py::bytes& b, int version) -> py::object {
    std::string_view sv = b;
    mqtt::Packet pk;
    const size_t used = mqtt::parse_packet(reinterpret_cast<const uint8_t*>(sv.data()), sv.size(), pk);
    if (!used) return py::none();
    py::dict d;
    d["type"] = (int)pk.type;
    d["flags"] = (int)pk.flags;
    d["size"] = used;
    d["body"] = py::bytes(pk.body);
    if (pk.type == mqtt::PUBLISH) {
      mqtt::Message msg = mqtt::decode_publish(pk, version);
      d["topic"] = msg.topic;
      d["payload"] = py::bytes(msg.payload);
      d["qos"] = msg.qos;
      d["retain"] = msg.retain;
      d["packet_id"] = (int)msg.packet_id;
    }
    return d;
  }, py::arg("data"), py::arg("version") = 5);

  py::class_<mqtt::Broker>(m, "MqttBroker")
      .def(py::init([](int port, const std::string& user, const std::string& pw, int max_qos,
                       const std::string& kafka_bootstrap, const py::list& mappings, const std::string& k_mech,
                       const std::string& k_user, const std::string& k_pw, int batch, int linger_ms) {
             mqtt::BrokerConfig c;
             c.port = port;
             c.username = user;
             c.password = pw;
             c.max_qos = max_qos;
             c.kafka_bootstrap = kafka_bootstrap;
             c.kafka.client_id = "mqtt-kafka-bridge";
             c.kafka.sasl_mechanism = k_mech;
             c.kafka.sasl_username = k_user;
             c.kafka.sasl_password = k_pw;
             c.bridge_batch = batch;
             c.bridge_linger_ms = linger_ms;
             for (auto item : mappings) {
               auto t = item.cast<py::tuple>();  // (id, [filters], kafka_topic)
               mqtt::TopicMapping tm;
               tm.id = t[0].cast<std::string>();
               tm.filters = t[1].cast<std::vector<std::string>>();
               tm.kafka_topic = t[2].cast<std::string>();
               c.mappings.push_back(tm);
             }
             py::gil_scoped_release rel;
             return new mqtt::Broker(c);
           }),
           py::arg("port") = 0, py::arg("username") = "", py::arg("password") = "", py::arg("max_qos") = 2,
           py::arg("kafka_bootstrap") = "", py::arg("mappings") = py::list(), py::arg("kafka_sasl_mechanism") = "",
           py::arg("kafka_sasl_username") = "", py::arg("kafka_sasl_password") = "", py::arg("bridge_batch") = 1024,
           py::arg("bridge_linger_ms") = 2)
      .def_property_readonly("port", &mqtt::Broker::port)
      .def("publish",
           [](mqtt::Broker& b, const std::string& topic, const py::bytes& payload, int qos, bool retain) {
             mqtt::Message msg;
             msg.topic = topic;
             msg.payload = payload;
             msg.qos = qos;
             msg.retain = retain;
             py::gil_scoped_release rel;
             b.publish(msg);
           },
           py::arg("topic"), py::arg("payload"), py::arg("qos") = 0, py::arg("retain") = false)
      .def("stats", [](mqtt::Broker& b) {
        const auto st = b.stats();
        py::dict d;
        d["incoming_publish"] = st.incoming_publish;
        d["outgoing_publish"] = st.outgoing_publish;
        d["connections_current"] = st.connections_current;
        d["connections_total"] = st.connections_total;
        d["retained"] = st.retained;
        d["kafka_sent"] = st.kafka_sent;
        d["kafka_failed"] = st.kafka_failed;
        d["kafka_queued"] = st.kafka_queued;
        return d;
      })
      .def("mapping_counts", &mqtt::Broker::mapping_counts)
      .def("flush",
           [](mqtt::Broker& b, int timeout_ms) {
             py::gil_scoped_release rel;
             return b.flush(timeout_ms);
           },
           py::arg("timeout_ms") = 10000)
      .def("stop", [](mqtt::Broker& b) {
        py::gil_scoped_release rel;
        b.stop();
      });

  py::class_<mqtt::Client>(m, "MqttClient")
      .def(py::init<>())
      .def("connect",
           [](mqtt::Client& c, const std::string& host, int port, const std::string& cid, int version, int keepalive,
              bool clean, const std::string& user, const std::string& pw, int timeout_ms) {
             py::gil_scoped_release rel;
             return c.connect(host, port, cid, version, (uint16_t)keepalive, clean, user, pw, timeout_ms);
           },
           py::arg("host"), py::arg("port"), py::arg("client_id"), py::arg("version") = 5,
           py::arg("keepalive") = 60, py::arg("clean") = true, py::arg("username") = "", py::arg("password") = "",
           py::arg("timeout_ms") = 5000)
      .def("publish",
           [](mqtt::Client& c, const std::string& topic, const py::bytes& payload, int qos, bool retain) {
             std::string p = payload;
             py::gil_scoped_release rel;
             c.publish(topic, p, qos, retain);
           },
           py::arg("topic"), py::arg("payload"), py::arg("qos") = 0, py::arg("retain") = false)
      .def("subscribe",
           [](mqtt::Client& c, const std::vector<std::pair<std::string, int>>& f) {
             py::gil_scoped_release rel;
             return c.subscribe(f);
           })
      .def("unsubscribe",
           [](mqtt::Client& c, const std::vector<std::string>& f) {
             py::gil_scoped_release rel;
             c.unsubscribe(f);
           })
      .def("receive",
           [](mqtt::Client& c, int timeout_ms) -> py::object {
             mqtt::Message msg;
             bool ok;
             {
               py::gil_scoped_release rel;
               ok = c.receive(msg, timeout_ms);
             }
             if (!ok) return py::none();
             return py::make_tuple(msg.topic, py::bytes(msg.payload), msg.qos, msg.retain);
           },
           py::arg("timeout_ms") = 1000)
      .def("ping",
           [](mqtt::Client& c, int timeout_ms) {
             py::gil_scoped_release rel;
             return c.ping(timeout_ms);
           },
           py::arg("timeout_ms") = 2000)
      .def("disconnect",
           [](mqtt::Client& c) {
             py::gil_scoped_release rel;
             c.disconnect();
           })
      .def_property_readonly("connected", &mqtt::Client::connected)
      .def_property_readonly("session_present", &mqtt::Client::session_present);

  m.def("mqtt_simulate",
        [](const py::dict& d) {
          mqtt::SimConfig c;
          if (d.contains("host")) c.host = d["host"].cast<std::string>();
          if (d.contains("port")) c.port = d["port"].cast<int>();
          if (d.contains("client_prefix")) c.client_prefix = d["client_prefix"].cast<std::string>();
          if (d.contains("id_digits")) c.id_digits = d["id_digits"].cast<int>();
          if (d.contains("id_offset")) c.id_offset = d["id_offset"].cast<int>();
          if (d.contains("topic_prefix")) c.topic_prefix = d["topic_prefix"].cast<std::string>();
          if (d.contains("clients")) c.clients = d["clients"].cast<int>();
          if (d.contains("messages_per_client")) c.messages_per_client = d["messages_per_client"].cast<int>();
          if (d.contains("interval_s")) c.interval_s = d["interval_s"].cast<double>();
          if (d.contains("ramp_s")) c.ramp_s = d["ramp_s"].cast<double>();
          if (d.contains("qos")) c.qos = d["qos"].cast<int>();
          if (d.contains("version")) c.version = d["version"].cast<int>();
          if (d.contains("threads")) c.threads = d["threads"].cast<int>();
          if (d.contains("seed")) c.seed = d["seed"].cast<uint64_t>();
          if (d.contains("failure_rate")) c.failure_rate = d["failure_rate"].cast<double>();
          if (d.contains("username")) c.username = d["username"].cast<std::string>();
          if (d.contains("password")) c.password = d["password"].cast<std::string>();
          if (d.contains("lo")) c.lo = d["lo"].cast<std::vector<double>>();
          if (d.contains("hi")) c.hi = d["hi"].cast<std::vector<double>>();
          if (d.contains("is_int")) c.is_int = d["is_int"].cast<std::vector<int>>();
          if (d.contains("paced")) c.paced = d["paced"].cast<bool>();
          if (d.contains("start_at_unix")) c.start_at_unix = d["start_at_unix"].cast<double>();
          if (d.contains("stamp_ns")) c.stamp_ns = d["stamp_ns"].cast<bool>();
          if (d.contains("source_ips")) c.source_ips = d["source_ips"].cast<std::vector<std::string>>();
          mqtt::SimStats st;
          {
            py::gil_scoped_release rel;
            st = mqtt::simulate(c);
          }
          py::dict out;
          out["connected"] = st.connected;
          out["connect_failed"] = st.connect_failed;
          out["published"] = st.published;
          out["acked"] = st.acked;
          out["publish_failed"] = st.publish_failed;
          out["elapsed_s"] = st.elapsed_s;
          out["connect_s"] = st.connect_s;
          out["publish_s"] = st.publish_s;
          out["max_lag_ms"] = st.max_lag_ms;
          out["late_10ms"] = st.late_10ms;
          return out;
        },
        py::arg("config"));
  m.def("mqtt_car_payload", [](const py::dict& d, uint64_t car, uint64_t seq, int64_t ts) {
    mqtt::SimConfig c;
    if (d.contains("seed")) c.seed = d["seed"].cast<uint64_t>();
    if (d.contains("failure_rate")) c.failure_rate = d["failure_rate"].cast<double>();
    if (d.contains("lo")) c.lo = d["lo"].cast<std::vector<double>>();
    if (d.contains("hi")) c.hi = d["hi"].cast<std::vector<double>>();
    if (d.contains("is_int")) c.is_int = d["is_int"].cast<std::vector<int>>();
    return py::bytes(mqtt::car_payload_json(c, car, seq, ts));
  });
}
