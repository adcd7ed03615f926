/*
 * EngineReplayPreparation -- ReplayingState's decode work for one failed task in ONE engine
 * call (nReplayPrepare -> clg_replay_prepare): the main log for the LogReplayer and every
 * subpartition recovery buffer for its SubpartitionRecoveryThread
 * (ReplayingState.java:67-70, :108-214).
 *
 * The reference decodes the main log lazily, one determinant per replayed call
 * (LogReplayerImpl.deserializeNext, LogReplayerImpl.java:138-145), and each subpartition's
 * buffer in its own thread, one decodeNext per BufferBuilt determinant (:161-190).  Here one
 * batched decode on the GPU finds every record of the main log and turns every recovery
 * buffer into its list of buildAndLogBuffer sizes, plus the first record each thread would
 * fail on.  The objects and exceptions stay the reference's:
 *   * mainLog(log) is an EngineDecodedLog whose next() materialises each determinant with
 *     the reference's per-type reader and, from the first bad record on, hands over to the
 *     reference's decodeNext (LogReplayerImpl patch, INTEGRATION.md);
 *   * sizes(partition, index) gives a recovery thread its sizes and where to put the
 *     buffer's readerIndex afterwards: at the first bad record, whose decodeNext then throws
 *     exactly what the reference throws, or at the end (ReplayingState patch, INTEGRATION.md).
 *
 * The task's subpartitions are taken in context.subpartitionTable.cellSet() order, as
 * createSubpartitionRecoveryThreads iterates them.  Source-only: this container has no JDK.
 */
package org.apache.flink.runtime.causal.recovery;

import org.apache.flink.runtime.causal.DeterminantResponseEvent;
import org.apache.flink.runtime.causal.engine.ClonosEngine;
import org.apache.flink.runtime.causal.engine.EngineDecodedLog;
import org.apache.flink.runtime.causal.log.job.CausalLogID;
import org.apache.flink.runtime.io.network.partition.PipelinedSubpartition;
import org.apache.flink.runtime.jobgraph.IntermediateResultPartitionID;
import org.apache.flink.shaded.guava18.com.google.common.collect.Table;
import org.apache.flink.shaded.netty4.io.netty.buffer.ByteBuf;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.HashMap;
import java.util.Map;

import static org.apache.flink.runtime.causal.engine.ClonosEngine.*;

public final class EngineReplayPreparation {

	/** A recovery thread's work: sizes[0, count) for buildAndLogBuffer, then the buffer's
	 *  readerIndex goes to resumeAt (the first bad record, or the end). */
	public static final class SubpartitionSizes {
		private final ByteBuffer sizes;
		private final int first;
		private final int count;
		private final int resumeAt;

		SubpartitionSizes(ByteBuffer sizes, int first, int count, int resumeAt) {
			this.sizes = sizes;
			this.first = first;
			this.count = count;
			this.resumeAt = resumeAt;
		}

		public int count() {
			return count;
		}

		public int get(int k) {
			return sizes.getInt(4 * (first + k));
		}

		public int resumeAt() {
			return resumeAt;
		}
	}

	private final RecoveryManagerContext context;
	private final ByteBuffer recOff;
	private final ByteBuffer tag;
	private final long[] mainResult = new long[6];
	private final Map<IntermediateResultPartitionID, Map<Integer, SubpartitionSizes>> bySubpartition = new HashMap<>();

	public EngineReplayPreparation(ClonosEngine engine, RecoveryManagerContext context,
								   DeterminantResponseEvent determinantAccumulator) {
		this.context = context;
		final short vertex = context.getTaskVertexID().getVertexID();
		final Map<CausalLogID, ByteBuf> dets = determinantAccumulator.getDeterminants();
		final Table<IntermediateResultPartitionID, Integer, PipelinedSubpartition> table = context.subpartitionTable;
		final int ns = table.size();
		final ByteBuffer[] bufs = new ByteBuffer[ns + 1];
		final ByteBuf[] held = new ByteBuf[ns + 1];
		final int[] lens = new int[ns + 1];
		final long[] subs = new long[3 * ns];
		held[0] = dets.get(new CausalLogID(context.getTaskVertexID()));
		CausalLogID id = new CausalLogID(vertex);
		int j = 0;
		long sizeSlots = 0;
		for (Table.Cell<IntermediateResultPartitionID, Integer, PipelinedSubpartition> cell : table.cellSet()) {
			final IntermediateResultPartitionID p = cell.getRowKey();
			final byte index = cell.getColumnKey().byteValue();
			id.replace(p.getLowerPart(), p.getUpperPart(), index); // as createSubpartitionRecoveryThreads
			held[1 + j] = dets.get(id);
			subs[3 * j] = p.getLowerPart();
			subs[3 * j + 1] = p.getUpperPart();
			subs[3 * j + 2] = index;
			j++;
		}
		for (int i = 0; i <= ns; i++) {
			if (held[i] == null) {
				continue;
			}
			lens[i] = held[i].readableBytes();
			bufs[i] = direct(held[i]);
			if (i > 0) {
				sizeSlots += lens[i] / 5;
			}
		}
		final int mainLen = lens[0];
		final int cap = mainLen / 2 + 1, wcap = mainLen / 6 + 1;
		this.recOff = ByteBuffer.allocateDirect(4 * cap).order(ByteOrder.nativeOrder());
		this.tag = ByteBuffer.allocateDirect(cap);
		final ByteBuffer v0 = ByteBuffer.allocateDirect(8 * cap);
		final ByteBuffer wIdx = ByteBuffer.allocateDirect(4 * wcap), wRc = ByteBuffer.allocateDirect(4 * wcap);
		final ByteBuffer wV1 = ByteBuffer.allocateDirect(8 * wcap), wVo = ByteBuffer.allocateDirect(4 * wcap);
		final ByteBuffer wVl = ByteBuffer.allocateDirect(4 * wcap), wSub = ByteBuffer.allocateDirect(wcap);
		final ByteBuffer sizes = ByteBuffer.allocateDirect((int) Math.max(4, 4 * sizeSlots)).order(ByteOrder.nativeOrder());
		final long[] subRes = new long[5 * Math.max(1, ns)];
		final int st = nReplayPrepare(engine.handle(), vertex, bufs, lens, subs, recOff, tag, v0, wIdx, wRc, wV1, wVo,
			wVl, wSub, mainResult, sizes, subRes);
		if (st != CLG_OK && mainResult[2] == CLG_OK) {
			check(st); // an engine failure, not a decode error of the main log
		}
		j = 0;
		for (Table.Cell<IntermediateResultPartitionID, Integer, PipelinedSubpartition> cell : table.cellSet()) {
			final int count = (int) subRes[5 * j];
			final int status = (int) subRes[5 * j + 1];
			final int resume = status == CLG_OK ? lens[1 + j] : (int) subRes[5 * j + 2];
			bySubpartition.computeIfAbsent(cell.getRowKey(), k -> new HashMap<>())
				.put(cell.getColumnKey(), new SubpartitionSizes(sizes, (int) subRes[5 * j + 4], count, resume));
			j++;
		}
	}

	/** The main log's records for LogReplayerImpl (null when the response holds no main log). */
	public EngineDecodedLog mainLog(ByteBuf log) {
		if (log == null) {
			return null;
		}
		return new EngineDecodedLog(log, context.causalLog.getDeterminantEncoder(), recOff, tag, (int) mainResult[0],
			(int) mainResult[2], (int) mainResult[4]);
	}

	/** The sizes the recovery thread of (partition, index) builds buffers with. */
	public SubpartitionSizes sizes(IntermediateResultPartitionID partition, int index) {
		final Map<Integer, SubpartitionSizes> m = bySubpartition.get(partition);
		return m == null ? null : m.get(index);
	}

	private static ByteBuffer direct(ByteBuf b) {
		if (b.isDirect() && b.nioBufferCount() == 1) {
			return b.nioBuffer(b.readerIndex(), b.readableBytes());
		}
		final ByteBuffer copy = ByteBuffer.allocateDirect(Math.max(1, b.readableBytes()));
		copy.put(b.nioBuffer(b.readerIndex(), b.readableBytes()));
		copy.flip();
		return copy;
	}
}
