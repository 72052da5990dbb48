// rtdump.h — tiny named-array container used by the oracle tools to exchange golden
// vectors with the Python tests (reader: tests/rtdump.py).  TEST INFRASTRUCTURE ONLY.
//
// Layout: "RTD1", then records {u32 name_len, name, u8 dtype, u8 ndim, u64 shape[ndim],
// raw little-endian data}, terminated by name_len == 0.
// dtype: 'f' f32, 'd' f64, 'i' i32, 'I' u32, 'q' i64, 'Q' u64, 'B' u8.
#pragma once
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

class RtDump {
public:
    explicit RtDump(const std::string &path) {
        f_ = std::fopen(path.c_str(), "wb");
        if (!f_) throw std::runtime_error("rtdump: cannot open " + path);
        std::fwrite("RTD1", 1, 4, f_);
    }
    ~RtDump() { close(); }
    void close() {
        if (!f_) return;
        uint32_t z = 0;
        std::fwrite(&z, 4, 1, f_);
        std::fclose(f_);
        f_ = nullptr;
    }
    template <class T>
    void put(const std::string &name, const std::vector<T> &v, std::vector<uint64_t> shape = {}) {
        if (shape.empty()) shape.push_back(v.size());
        put_raw(name, code<T>(), shape, v.data(), v.size() * sizeof(T));
    }
    template <class T>
    void scalar(const std::string &name, T v) { put_raw(name, code<T>(), {1}, &v, sizeof(T)); }

private:
    template <class T> static char code();
    void put_raw(const std::string &name, char dt, const std::vector<uint64_t> &shape, const void *p, size_t n) {
        uint32_t len = (uint32_t)name.size();
        std::fwrite(&len, 4, 1, f_);
        std::fwrite(name.data(), 1, len, f_);
        uint8_t d = (uint8_t)dt, nd = (uint8_t)shape.size();
        std::fwrite(&d, 1, 1, f_);
        std::fwrite(&nd, 1, 1, f_);
        std::fwrite(shape.data(), 8, shape.size(), f_);
        if (n) std::fwrite(p, 1, n, f_);
    }
    std::FILE *f_ = nullptr;
};
template <> inline char RtDump::code<float>() { return 'f'; }
template <> inline char RtDump::code<double>() { return 'd'; }
template <> inline char RtDump::code<int32_t>() { return 'i'; }
template <> inline char RtDump::code<uint32_t>() { return 'I'; }
template <> inline char RtDump::code<int64_t>() { return 'q'; }
template <> inline char RtDump::code<uint64_t>() { return 'Q'; }
template <> inline char RtDump::code<uint8_t>() { return 'B'; }
