/*
 * HipShardedKnnFunction -- PointPointKNNQuery.windowBased (PointPointKNNQuery.java:132-201) over
 * the GPUs of one node: each subtask (= rank = GPU) evaluates its cell-column band of every window
 * on its device, and the windowAll merge (:195-200, KNNQuery.java:213-272) becomes an RCCL
 * all-gather of the bands' top-k records plus the same top-k-distinct merge on every GPU -- the
 * collective behind the C ABI (gf_knn_exchange_strings_batch), batched over B windows.  NOT
 * COMPILED here (no JDK in the build image); see INTEGRATION.md and tests/test_shim_native.py
 * (test_java_call_sequences drives this class's native sequence through the C core on the GPU).
 *
 *   env.setMaxParallelism(M);
 *   CellColumnBands bands = new CellColumnBands(gridArgs, nranks, M);
 *   pointStream.union(heartbeats)                       // CellColumnBands.marker(b) for every band
 *       .keyBy(bands)                                    // band b -> subtask b
 *       .window(SlidingProcessingTimeWindows.of(size, slide))
 *       .apply(new HipShardedKnnFunction(gridArgs, queryPoint, r, k, nranks, batch, dir, jobKey))
 *       .setParallelism(nranks)
 *       .keyBy(p -> p.windowEnd)
 *       .process(new ShardedKnnAssembler(k))            // -> Tuple3(start, end, PQ), as the reference
 *
 * Per window: the band's Points -> direct buffers (objID Strings interned per rank) ->
 * knnShardedEnqueue (the band's points are the window's global indices rank << 32 + position);
 * every B-th window the batch's records are exchanged by String (the ranks' dictionaries differ;
 * the merge dedupes by Point.objID as KNNQuery.java:232-251 does), and the batch's results are
 * read: every rank gets the whole window's top k, and emits the entries its band holds (owned)
 * with their merged ranks; the assembler puts the ranks' parts together.  B = 1 reads every window
 * right away (bounded inputs: a window function cannot emit after its last firing).
 *
 * Communicator: CommRendezvous (rank 0's 128-byte id through a shared directory, commCreate =
 * ncclCommInitRank on each subtask's context).
 */
package GeoFlink.native_;

import GeoFlink.spatialObjects.Point;
import org.apache.flink.configuration.Configuration;
import org.apache.flink.streaming.api.functions.windowing.RichWindowFunction;
import org.apache.flink.streaming.api.windowing.windows.TimeWindow;
import org.apache.flink.util.Collector;

import java.util.ArrayDeque;
import java.util.ArrayList;

public class HipShardedKnnFunction extends RichWindowFunction<Point, ShardedKnnPartial, Integer, TimeWindow> {

  private final double[] gridArgs;
  private final double qx, qy, radius;
  private final int k, nranks, batch;
  private final String rendezvousDir, jobKey;

  private transient int rank;
  private transient long ctx, plan, comm;
  private transient HipColumns cols;
  private transient double[] outDist;
  private transient long[] outIdx;
  private transient int[] owned;
  private transient ArrayDeque<Pending> pending;

  private static final class Pending {
    final long ticket, start, end;
    final ArrayList<Point> points;

    Pending(long ticket, long start, long end, ArrayList<Point> points) {
      this.ticket = ticket;
      this.start = start;
      this.end = end;
      this.points = points;
    }
  }

  public HipShardedKnnFunction(double[] gridArgs, Point queryPoint, double radius, int k, int nranks, int batch,
                               String rendezvousDir, String jobKey) {
    this.gridArgs = gridArgs.clone();
    this.qx = queryPoint.point.getX();
    this.qy = queryPoint.point.getY();
    this.radius = radius;
    this.k = k;
    this.nranks = nranks;
    this.batch = batch;
    this.rendezvousDir = rendezvousDir;
    this.jobKey = jobKey;
  }

  @Override
  public void open(Configuration parameters) throws Exception {
    rank = getRuntimeContext().getIndexOfThisSubtask();
    ctx = GeoFlinkHip.ctxCreate(rank);  // one GPU per subtask: device = rank on its node
    plan = GeoFlinkHip.knnPlan(ctx, gridArgs, qx, qy, radius, k);
    comm = CommRendezvous.create(ctx, nranks, rank, rendezvousDir, jobKey);
    GeoFlinkHip.knnShardedBegin(ctx, plan, comm, batch, 32L * k + 64);
    cols = new HipColumns(true);
    outDist = new double[k];
    outIdx = new long[k];
    owned = new int[k];
    pending = new ArrayDeque<>();
  }

  @Override
  public void close() {
    if (comm != 0) GeoFlinkHip.commDestroy(comm);
    if (plan != 0) GeoFlinkHip.knnPlanDestroy(plan);
    if (ctx != 0) GeoFlinkHip.ctxDestroy(ctx);
    comm = plan = ctx = 0;
  }

  @Override
  public void apply(Integer key, TimeWindow window, Iterable<Point> input, Collector<ShardedKnnPartial> out) {
    final ArrayList<Point> pts = new ArrayList<>();
    for (Point p : input)
      if (!CellColumnBands.isMarker(p)) pts.add(p);  // heartbeats only make the band fire
    cols.fill(ctx, pts);
    final long base = (long) rank << 32;
    final long ticket = GeoFlinkHip.knnShardedEnqueue(ctx, plan, cols.x, cols.y, cols.objID, pts.size(), base);
    pending.add(new Pending(ticket, window.getStart(), window.getEnd(), pts));
    if ((ticket + 1) % batch != 0) return;  // the batch's exchange is issued with its last window
    while (!pending.isEmpty()) {  // one host wait for the batch, then every window of it
      final Pending w = pending.poll();
      final int m = GeoFlinkHip.knnShardedResult(ctx, plan, w.ticket, outDist, outIdx, owned);
      final ShardedKnnPartial part = new ShardedKnnPartial(w.start, w.end, nranks, rank, m);
      for (int j = 0; j < m; j++)
        if (owned[j] != 0) part.add(j, w.points.get((int) (outIdx[j] - base)), outDist[j]);
      out.collect(part);
    }
  }
}
