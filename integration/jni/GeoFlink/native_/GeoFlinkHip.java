/*
 * GeoFlinkHip -- the Java side of the JNI shim that puts libgeoflink_hip.so behind the GeoFlink
 * window operators (see INTEGRATION.md).  NOT COMPILED in this repository: the build image has
 * no JDK (no javac, no jni.h).  It is kept as a real source file so a maintainer can drop it
 * next to the reference's operators (package GeoFlink.native_) and build it with the JDK.
 * tests/test_shim_native.py checks that every native here has its C function in geoflink_jni.c
 * with the JNI types of these parameters, and drives the C core each of them calls on the GPU.
 *
 * Every handle is a native pointer held in a long.  Window buffers are direct ByteBuffers in
 * native byte order (x, y: double; objID keys, ts: long).  A context (ctxCreate) is one Flink
 * subtask's device context plus the device buffers its windows reuse; plans cache their own
 * device windows, so a continuous query uploads into the same device buffers window after
 * window.  Nothing is shared between contexts.
 *
 * Anchors (what each native call replaces):
 *   objidIntern / objidDecode  Point.objID Strings (Point.java:41-47) <-> the int64 keys the
 *                device evaluates (include/geoflink_hip.h, "objID keys")
 *   knnWindow    PointPointKNNQuery.windowBased (PointPointKNNQuery.java:132-201) +
 *                KNNQuery.kNNWinAllEvaluationPointStream (KNNQuery.java:213-272)
 *   knnPolygonPlan  PointPolygonKNNQuery (PointPolygonKNNQuery.java:245-317)
 *   knnWindowSharded / knnSharded*  the windowAll merge (PointPointKNNQuery.java:198-200) across the
 *                GPUs of a node: an RCCL exchange of the bands' top-k records (HipShardedKnnFunction)
 *   knnSliding*  SlidingProcessingTimeWindows.of(size, slide) around the kNN apply
 *                (PointPointKNNQuery.java:158,198-200): panes evaluated once, windows merged
 *   rangeSliding*  the same apply under SlidingProcessingTimeWindows (PointPointRangeQuery.java:149)
 *   rangeWindow  PointPointRangeQuery.windowBased apply (PointPointRangeQuery.java:150-186),
 *                PointPolygonRangeQuery apply (PointPolygonRangeQuery.java:170-204)
 *   joinWindow   JoinQuery.getReplicatedPointQueryStream (JoinQuery.java:73-90) +
 *                PointPointJoinQuery.windowBased (PointPointJoinQuery.java:148-182)
 *   polygonJoinWindow  JoinQuery.java:93-115 + PointPolygonJoinQuery.java:154-213
 *   csvParse     Deserialization.CSVTSVToTSpatial.map (Deserialization.java:291-325)
 *   geoJsonParse Deserialization.GeoJSONToTSpatial(uGrid, dateFormat, propertyTimeStamp,
 *                propertyObjID).map (Deserialization.java:64-70,149-211), Point geometries
 */
package GeoFlink.native_;

import java.nio.ByteBuffer;
import java.nio.charset.StandardCharsets;

public final class GeoFlinkHip {
  static { System.loadLibrary("geoflink_jni"); }   // libgeoflink_jni.so -> libgeoflink_hip.so

  private GeoFlinkHip() {}

  /** objID key of a null String (a GeoJSON feature without the objID property). */
  public static final long OBJID_NULL = Long.MAX_VALUE;

  // one context per Flink subtask (RichAllWindowFunction.open / close)
  public static native long ctxCreate(int device);
  public static native void ctxDestroy(long ctx);

  // ---- objID Strings <-> keys (the context's dictionary) ------------------------------------
  // String i = UTF-8 bytes[offs[i], offs[i+1]) (offs: n + 1 entries) -> keys[i]
  public static native void objidIntern(long ctx, byte[] bytes, long[] offs, int n, long[] keys);
  // keys -> the Strings' UTF-8 bytes; offs (n + 1 entries) filled
  public static native byte[] objidDecode(long ctx, long[] keys, int n, long[] offs);

  /** Point.objID Strings of a window -> keys (null -> OBJID_NULL) */
  public static long[] intern(long ctx, String[] objIDs, int n) {
    byte[][] enc = new byte[n][];
    long[] offs = new long[n + 1];
    for (int i = 0; i < n; i++) {
      enc[i] = objIDs[i] == null ? new byte[0] : objIDs[i].getBytes(StandardCharsets.UTF_8);
      offs[i + 1] = offs[i] + enc[i].length;
    }
    byte[] bytes = new byte[(int) offs[n]];
    for (int i = 0; i < n; i++) System.arraycopy(enc[i], 0, bytes, (int) offs[i], enc[i].length);
    long[] keys = new long[n];
    objidIntern(ctx, bytes, offs, n, keys);
    for (int i = 0; i < n; i++) if (objIDs[i] == null) keys[i] = OBJID_NULL;
    return keys;
  }

  /** result keys -> Point.objID Strings (UTF-8, not JNI's modified UTF-8) */
  public static String[] decode(long ctx, long[] keys, int n) {
    long[] offs = new long[n + 1];
    byte[] bytes = objidDecode(ctx, keys, n, offs);
    String[] out = new String[n];
    for (int i = 0; i < n; i++)
      out[i] = keys[i] == OBJID_NULL ? null
             : new String(bytes, (int) offs[i], (int) (offs[i + 1] - offs[i]), StandardCharsets.UTF_8);
    return out;
  }

  // ---- kNN ----------------------------------------------------------------------------------
  // grids as double[] {n, minX, maxX, minY, maxY} (UniformGrid(n, minX, maxX, minY, maxY))
  // pinned host memory as a direct ByteBuffer (native order is the caller's): a kNN window's
  // objID column placed here is read in place by the kernels (16 B per point over PCIe, not 24);
  // free it with pinnedFree, never let the GC drop it while a window may still read it
  public static native ByteBuffer pinnedBuffer(long bytes);
  public static native void pinnedFree(ByteBuffer buf);
  public static native long knnPlan(long ctx, double[] grid, double qx, double qy, double r, int k);
  // polygons as CSR: ringOff[npoly+1] into vertOff, vertOff[nrings+1] into vx / vy (closed rings)
  public static native long knnPolygonPlan(long ctx, double[] grid, int[] ringOff, int[] vertOff, double[] vx,
                                           double[] vy, double r, int k, boolean approximate);
  public static native void knnPlanDestroy(long plan);
  // x, y, objID keys of one window (ts is not read by window evaluation); returns the number of
  // neighbours written to out* (ascending (dist, objID)), outIdx = the window-local indices;
  // out* hold at least k entries
  public static native int knnWindow(long ctx, long plan, ByteBuffer x, ByteBuffer y, ByteBuffer objID, int n,
                                     long[] outObjID, double[] outDist, long[] outIdx, int k);

  // ---- multi-GPU kNN: one subtask per GPU holds its cell-column band of every window; the
  // windowAll merge (PointPointKNNQuery.java:198-200) is an RCCL exchange of the bands' top-k
  // records.  One TaskManager per GPU: rank 0's commUniqueId() is broadcast to every subtask
  // (a broadcast stream / the job configuration), each calls commCreate on its context (blocks
  // until all ranks joined); one TaskManager holding every GPU: commCreateAll(devices).
  public static native byte[] commUniqueId();
  public static native long commCreate(long ctx, byte[] id, int nranks, int rank);
  public static native long[] commCreateAll(int[] devices);
  public static native void commDestroy(long comm);
  // this subtask's band (its points are the window's global indices indexBase ..
  // indexBase + n - 1) -> the WHOLE window's neighbours, identical on every rank; every rank calls
  // it once per window, in the same order
  public static native int knnWindowSharded(long ctx, long plan, long comm, ByteBuffer x, ByteBuffer y,
                                            ByteBuffer objID, int n, long indexBase, long[] outObjID,
                                            double[] outDist, long[] outIdx, int k);
  // The batched, asynchronous form (HipShardedKnnFunction; the path bench.py --gpus N times):
  // knnShardedEnqueue queues this subtask's band of a window and returns its ticket; every
  // batch-th enqueue issues ONE exchange of the batch's records by String (every rank must make
  // the same calls in the same order); knnShardedResult(ticket) then gives the window's merged
  // neighbours -- outDist, outIdx (global: indexBase + band position) and owned[j] = 1 for this
  // band's Points -- and frees the ticket's slot (read a ticket before enqueueing 2 * batch more).
  // knnShardedFlush exchanges an incomplete batch (end of input).  capBytes bounds the objID
  // Strings of one record (e.g. 32 * k).
  public static native void knnShardedBegin(long ctx, long plan, long comm, int batch, long capBytes);
  public static native long knnShardedEnqueue(long ctx, long plan, ByteBuffer x, ByteBuffer y, ByteBuffer objID,
                                              int n, long indexBase);
  public static native void knnShardedFlush(long ctx, long plan);
  public static native int knnShardedResult(long ctx, long plan, long ticket, double[] outDist, long[] outIdx,
                                            int[] owned);

  // ---- sliding kNN (pane engine) ---------------------------------------------------------
  // size / gcd(size, slide) <= 64; the plan must outlive the sliding handle
  public static native long knnSlidingCreate(long ctx, long plan, long sizeMs, long slideMs);
  public static native void knnSlidingDestroy(long sliding);
  // pane p holds timestamps [p * paneMs, (p + 1) * paneMs)
  public static native long knnSlidingPaneMs(long sliding);
  // push pane `pane` (consecutive indices; an empty pane with n = 0); returns the end (ms) of
  // the window it closed, or -1.  Decode a closed window within the next 8 windows.
  public static native long knnSlidingPush(long ctx, long sliding, long pane, ByteBuffer x, ByteBuffer y,
                                           ByteBuffer objID, int n);
  // a closed window's neighbours; outIdx = the point's position in the pushed stream
  public static native int knnSlidingDecode(long ctx, long sliding, long windowEnd, long[] outObjID,
                                            double[] outDist, long[] outIdx, int k);

  // ---- range ---------------------------------------------------------------------------
  public static native long rangePlan(long ctx, double[] grid, double[] qx, double[] qy, double r,
                                      boolean approximate);
  public static native long rangePolygonPlan(long ctx, double[] grid, int[] ringOff, int[] vertOff, double[] vx,
                                             double[] vy, double r, boolean approximate);
  public static native void rangePlanDestroy(long plan);
  // emitted point indices, ascending, into out (a direct int buffer of outCap entries); returns
  // their count -- larger than outCap: call again with a larger buffer
  public static native long rangeWindow(long ctx, long plan, ByteBuffer x, ByteBuffer y, int n, ByteBuffer out,
                                        int outCap);
  // approximate point queries with |Q| > 1: the points of the last rangeWindow that the reference
  // emits once per query point (PointPointRangeQuery.java:158-161) -- a subset of its list,
  // ascending; same count / capacity convention; 0 for other plans
  public static native long rangeWindowMulti(long ctx, long plan, ByteBuffer out, int outCap);

  // ---- sliding range (pane engine) ---------------------------------------------------------
  // SlidingProcessingTimeWindows.of(size, slide) around the range apply (PointPointRangeQuery.java:
  // 149-186): each pane evaluated once; plan from rangePlan / rangePolygonPlan (outlives this)
  public static native long rangeSlidingCreate(long ctx, long plan, long sizeMs, long slideMs);
  public static native void rangeSlidingDestroy(long sliding);
  public static native long rangeSlidingPaneMs(long sliding);
  // push pane `pane` (consecutive; empty with n = 0): the emitted points of the window it closed
  // (positions in the window's panes concatenated, ascending), windowEnd[0] = its end; null when
  // no window holding a point closed
  public static native int[] rangeSlidingPush(long ctx, long sliding, long pane, ByteBuffer x, ByteBuffer y, int n,
                                              long[] windowEnd);

  // ---- joins ---------------------------------------------------------------------------
  // pairs (ordinary / point index, query / polygon index) flattened
  public static native long[] joinWindow(long ctx, double[] uGrid, double[] qGrid, ByteBuffer ox, ByteBuffer oy,
                                         int no, ByteBuffer qx, ByteBuffer qy, int nq, double r,
                                         boolean approximate);
  public static native long[] polygonJoinWindow(long ctx, double[] grid, ByteBuffer x, ByteBuffer y, int n,
                                                int[] ringOff, int[] vertOff, double[] vx, double[] vy, double r,
                                                boolean approximate);

  // ---- ingest --------------------------------------------------------------------------
  // a chunk of complete lines -> x, y, objID keys, ts (direct buffers of capacity >= lines);
  // returns the number of points; objID Strings are interned in the context's dictionary.
  // A bad line throws (NumberFormatException / IllegalArgumentException naming the line).
  public static native int csvParse(long ctx, ByteBuffer text, int len, char delimiter, int[] schema /* objID, ts, x, y */,
                                    ByteBuffer x, ByteBuffer y, ByteBuffer objID, ByteBuffer ts, int capacity);
  // GeoJSONToTSpatial(uGrid, dateFormat, propertyTimeStamp, propertyObjID): dateFormat null
  // (integer ms) or "yyyy-MM-dd HH:mm:ss"; tzOffsetMinutes = TimeZone.getDefault().getRawOffset()
  // / 60000; valueLines: each line is the record's value instead of {"key":..,"value":..}
  public static native int geoJsonParse(long ctx, ByteBuffer text, int len, String propertyTimeStamp,
                                        String propertyObjID, String dateFormat, int tzOffsetMinutes,
                                        boolean valueLines, ByteBuffer x, ByteBuffer y, ByteBuffer objID,
                                        ByteBuffer ts, int capacity);
}
