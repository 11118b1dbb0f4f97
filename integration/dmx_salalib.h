// dmx_salalib.h -- reference-side binding: route salalib's makeGraph and VGA global to libdmx.so.
//
// A maintainer adds integration/dmx_salalib.cpp to salalib and calls these at the top of the two
// methods they accelerate (INTEGRATION.md shows the two-line hooks):
//   PointMap::sparkGraph2        salalib/pointdata.cpp:1246-1341
//   VGAVisualGlobal::run         salalib/vgamodules/vgavisualglobal.cpp:23-216
// Each returns true when the engine ran the analysis and `map` now holds exactly what the reference
// method would have left in it (the point states, nodes, attribute columns and statistics, through
// the reference's own PointMap::read of the engine's byte-identical PointMap::write image), and false
// when the map is outside what the engine reproduces exactly (no GPU, a grid set with a non-zero
// offset, merge links); the caller then runs its own code.  Cancellation through the Communicator
// throws Communicator::CancelledException as the reference does; engine errors throw
// depthmapX::RuntimeException.
#pragma once

class Communicator;
class PointMap;

namespace dmxsala {

bool sparkGraph2(PointMap& map, Communicator* comm, bool boundarygraph, double maxdist);
bool vgaVisualGlobal(PointMap& map, Communicator* comm, double radius, bool gates_only, bool simple_version);

// Test hooks (integration/bind_check.cpp): the PointMap <-> PointMap::write image conversions the two
// calls are built on.
bool saveMap(PointMap& map, void* bytes_out /* std::string* */);
bool loadMap(PointMap& map, const void* bytes /* const std::string* */);

}  // namespace dmxsala
