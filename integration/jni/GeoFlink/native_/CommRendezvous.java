/*
 * CommRendezvous -- the RCCL communicator of a multi-GPU kNN job (HipShardedKnnFunction): rank 0
 * draws the 128-byte unique id (commUniqueId = ncclGetUniqueId) and publishes it through a
 * directory every subtask of the node can read (written under a temporary name, then renamed: a
 * reader sees the whole id or nothing); every rank then calls commCreate (ncclCommInitRank, which
 * blocks until all nranks joined).  One TaskManager per GPU or one holding all of them: either
 * way each subtask thread drives its own GPU's communicator.  NOT COMPILED here (no JDK).
 */
package GeoFlink.native_;

import java.io.IOException;
import java.nio.file.Files;
import java.nio.file.Path;
import java.nio.file.Paths;
import java.nio.file.StandardCopyOption;

final class CommRendezvous {
  private CommRendezvous() {}

  static long create(long ctx, int nranks, int rank, String dir, String jobKey) throws IOException, InterruptedException {
    final Path id = Paths.get(dir, jobKey + ".gfcomm");
    byte[] bytes;
    if (rank == 0) {
      bytes = GeoFlinkHip.commUniqueId();
      final Path tmp = Files.createTempFile(Paths.get(dir), jobKey, ".tmp");
      Files.write(tmp, bytes);
      Files.move(tmp, id, StandardCopyOption.ATOMIC_MOVE, StandardCopyOption.REPLACE_EXISTING);
    } else {
      final long deadline = System.currentTimeMillis() + 120_000;
      while (!Files.exists(id)) {
        if (System.currentTimeMillis() > deadline) throw new IOException("no communicator id at " + id);
        Thread.sleep(20);
      }
      bytes = Files.readAllBytes(id);
    }
    return GeoFlinkHip.commCreate(ctx, bytes, nranks, rank);
  }
}
