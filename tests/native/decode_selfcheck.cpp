// Host build of point_decode.h for tests/test_point_decode.py: argv[1] = format (0 WKB, 1 WKT,
// 2 hex WKB); reads one row per stdin line, the row's raw bytes given as hex, and prints
// "<status> <x bits hex> <y bits hex>" per row.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "../../mosaic_amd/csrc/point_decode.h"

int main(int argc, char** argv) {
    const int fmt = argc > 1 ? atoi(argv[1]) : 1;
    std::string line;
    std::vector<uint8_t> row;
    while (std::getline(std::cin, line)) {
        row.resize(line.size() / 2);
        for (size_t k = 0; k < row.size(); k++) row[k] = (uint8_t)strtoul(line.substr(2 * k, 2).c_str(), nullptr, 16);
        double x = 0, y = 0;
        int rc = mosaic::decode::decode_row(fmt, row.data(), (int64_t)row.size(), &x, &y);
        uint64_t bx, by;
        memcpy(&bx, &x, 8);
        memcpy(&by, &y, 8);
        printf("%d %016llx %016llx\n", rc, (unsigned long long)bx, (unsigned long long)by);
    }
    return 0;
}
