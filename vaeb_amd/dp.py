"""Row partition of a global minibatch over data-parallel ranks.

The SGVB objective is a sum over batch rows (VAEB.py:340-344), so a step shards by rows:
rank r takes a contiguous block of the global minibatch and the gradients are summed with
one all-reduce.  Weak scaling gives every rank B rows (B_global = B * world); strong
scaling splits a fixed global batch as evenly as possible, earlier ranks taking the
remainder (100 over 8 ranks = 13,13,13,13,12,12,12,12)."""


def row_split(batch, world, rank, scaling="weak"):
    """Returns (rows of this rank, its row offset inside the global minibatch, B_global)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    if scaling == "weak":
        return batch, rank * batch, batch * world
    if scaling != "strong":
        raise ValueError(f"unknown scaling {scaling!r}")
    if batch < world:
        raise ValueError(f"strong scaling needs at least one row per rank ({batch} rows, {world} ranks)")
    base, extra = divmod(batch, world)
    rows = [base + (1 if r < extra else 0) for r in range(world)]
    return rows[rank], sum(rows[:rank]), batch
