// xml_loader.cpp -- Mitsuba 3 XML scene subset (Source/SceneXMLLoading.cpp).
// Round-1 placeholder: the OBJ path (config 1/2) is the measured workload; the
// XML loader is the next host row and reports a clear error.
#include <cstdio>

#include "scene.h"

namespace dcrt {

void SetLastError(const std::string& s);

bool LoadMitsubaXML(CScene* /*scene*/, const std::string& path)
{
    SetLastError("Mitsuba XML loading is not implemented yet: " + path);
    std::fprintf(stderr, "dcrt: Mitsuba XML loading is not implemented yet (%s)\n", path.c_str());
    return false;
}

}  // namespace dcrt
