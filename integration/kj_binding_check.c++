// kj_binding_check.c++ -- compile check of integration/kj_binding.h against the reference's own
// capnp / kj headers (tests/test_integration.py compiles it to an object file; nothing here
// runs).  It uses the binding the way the reference's callers use the packed API
// (samples/addressbook.c++:75,79; serialize-packed-test.c++:348-371).
#include "kj_binding.h"

#include <capnp/serialize.h>

void cpk_kj_binding_check(kj::BufferedOutputStream& out, kj::BufferedInputStream& in, int fd);

void cpk_kj_binding_check(kj::BufferedOutputStream& out, kj::BufferedInputStream& in, int fd) {
  capnp::MallocMessageBuilder builder;
  builder.initRoot<capnp::AnyPointer>();
  cpk_kj::writePackedMessage(out, builder);
  cpk_kj::writePackedMessageToFd(fd, builder);

  cpk_kj::PackedMessageReader reader(in);
  auto root = reader.getRoot<capnp::AnyPointer>();
  (void)root;
  capnp::MessageReader& generic = reader;  // usable wherever a MessageReader is expected
  (void)generic.getOptions();

  kj::byte packed[2] = {0, 0};
  (void)cpk_kj::computeUnpackedSizeInWords(kj::arrayPtr(packed, 2));
}
