// TEST INFRASTRUCTURE -- never part of the product, never measured.
//
// The reference's XML parse (Source/SceneXMLLoading.cpp:1044-1056: the file read into a
// char vector with a terminating NUL, xml_document<>::parse<parse_non_destructive>) with its
// UNMODIFIED vendored RapidXml (RapidXml/rapidxml.hpp, compiled from /root/reference by
// oracle/ref_xml/Makefile), and the element / attribute tree its value-graph walk reads
// (:247-581: element nodes through first_node / next_sibling, attributes by name, values as
// written -- non-destructive: no entity translation), serialised as the product's
// dcrt_xml_dump_tree does. tests/test_xml_pin.py compares the two.
#include "RapidXml/rapidxml.hpp"

#include <cstdint>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

namespace {

void Dump(const rapidxml::xml_node<>* parent, std::string* out)
{
    for (const rapidxml::xml_node<>* n = parent->first_node(); n; n = n->next_sibling()) {
        if (n->type() != rapidxml::node_element) continue;
        *out += "E" + std::string(n->name(), n->name_size()) + "\n";
        for (const rapidxml::xml_attribute<>* a = n->first_attribute(); a; a = a->next_attribute())
            *out += "A" + std::string(a->name(), a->name_size()) + "=" + std::string(a->value(), a->value_size()) + "\n";
        Dump(n, out);
        *out += "/\n";
    }
}

}  // namespace

extern "C" int refxml_dump_tree(const char* path, char* out, uint32_t capacity, uint32_t* outLength)
{
    std::ifstream in(path);
    if (!in) return -4;
    std::vector<char> xml((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    xml.emplace_back('\0');
    std::string dump;
    try {
        rapidxml::xml_document<> doc;
        doc.parse<rapidxml::parse_non_destructive>(xml.data());
        Dump(&doc, &dump);
    } catch (const rapidxml::parse_error&) {
        return -1;
    }
    *outLength = (uint32_t)dump.size();
    if (out && capacity) std::memcpy(out, dump.data(), dump.size() < capacity ? dump.size() : capacity);
    return dump.size() <= capacity ? 0 : -5;
}
