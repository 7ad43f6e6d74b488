// Host-runtime bindings (codec, Kafka, engine) — filled in as those subsystems land.
#include <pybind11/pybind11.h>

namespace py = pybind11;

namespace gale {
void bind_host(py::module_& m) { (void)m; }
}  // namespace gale
